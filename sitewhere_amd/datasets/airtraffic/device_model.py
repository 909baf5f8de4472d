# Air-traffic dataset: device management initializer (reference
# datasets/airtraffic/scripts/device-management/content/initializer/deviceModel.groovy): airlines,
# an airport area with its airspace and a restricted zone, aircraft tracker device types with
# commands, transport groups, and one tracker per aircraft with a flight path (positions,
# engine measurements and overheat alerts).

import math
import time

db, eb = device_builder, event_builder
now = int(time.time() * 1000)
airspace = [(34.0, -85.0), (34.0, -83.8), (33.3, -83.8), (33.3, -85.0)]
restricted = [(33.66, -84.46), (33.66, -84.40), (33.62, -84.40), (33.62, -84.46)]

db.persist(db.new_customer_type("airline", "Airline Company").with_description("A commercial airline."))
for tok, name in (("american", "American Airlines, Inc."), ("southwest", "Southwest Airlines Co."),
                  ("delta", "Delta Air Lines"), ("united", "United Airlines")):
    db.persist(db.new_customer("airline", None, tok, name))
db.persist(db.new_area_type("airport-type", "Air Port Type").with_description("An airport and its airspace."))
area = db.new_area("airport-type", None, "atl-airspace", "ATL airspace")
for lat, lon in airspace:
    area.coord(lat, lon)
db.persist(area)
zone = db.new_zone("atl-restricted", "Restricted", "atl-airspace").with_border_color("#aa0000") \
    .with_fill_color("#ff0000").with_opacity(0.3)
for lat, lon in restricted:
    zone.coord(lat, lon)
db.persist(zone)

ns = "http://sitewhere/common"
for tok, name in (("aircraft-tracker", "Aircraft Tracker"), ("airtraffic-plane", "Air Traffic Plane")):
    db.persist(db.new_device_type(tok, name).with_description(name + " reporting position and engine data."))
    for cmd in ("ping", "testEvents"):
        db.persist(db.new_command(tok, f"{tok}-{cmd}", ns, cmd).with_description("Verify the device can be reached."))
heavy = db.persist(db.new_group("heavy-transport", "Heavy Transport").with_role("heavy-transport").with_role("heavy"))
personal = db.persist(db.new_group("personal-transport", "Personal Transport").with_role("personal-transport")
                      .with_role("personal"))

members = {"heavy": [], "personal": []}
airlines = ["american", "southwest", "delta", "united"]
for i in range(params["flights"]):
    tok = f"flight-{i:03d}"
    dev = db.persist(db.new_device("aircraft-tracker", tok).with_comment(f"Tracker of aircraft-{i:03d}"))
    asg = db.persist(db.new_assignment(tok, airlines[i % 4], "atl-airspace", f"aircraft-{i:03d}"))
    members["heavy" if i % 3 else "personal"].append(db.new_group_element(tok))
    # a great-circle-ish straight path across the airspace, one position every ~20 s
    t = now - 3600 * 1000
    heading = rnd.random() * 2 * math.pi
    lat, lon = 33.65 + rnd.random() * 0.2, -84.4 + rnd.random() * 0.2
    locs, mx, alerts = [], [], []
    temp = 400.0
    for k in range(params["positions_per_flight"]):
        lat += 0.01 * math.cos(heading)
        lon += 0.01 * math.sin(heading)
        locs.append(eb.new_location(lat, lon, 9000.0 + 50 * k).on(t).track_state())
        temp = round(temp + rnd.random() * 20 - 8, 2)
        mx.append(eb.new_measurements().measurement("engine.temperature", temp).on(t).track_state())
        if temp > 560:
            alerts.append(eb.new_alert("engine.overheat", "Engine temperature high.").warning().on(t).track_state())
        t += 20000 + int(rnd.random() * 5000)
    ev = eb.for_assignment(asg)
    ev.persist_locations(locs)
    ev.persist_measurements(mx)
    ev.persist_alerts(alerts)
db.persist(db.new_group("heavy-transport", "Heavy Transport"), members["heavy"])
db.persist(db.new_group("personal-transport", "Personal Transport"), members["personal"])
