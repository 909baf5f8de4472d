# Construction-site dataset: device management initializer.
#
# Content of the reference's construction dataset
# (service-tenant-management/dockerimage/datasets/construction/scripts/device-management/content/
# initializer/deviceModel.groovy): a construction company with subcontractors, a region with a
# construction site and its work-area zone, the tracker / sensor / gateway device types (the gateway
# with a composite element schema) and their commands, three device groups, and devices assigned to
# site assets with two hours of history each -- fuel / engine-temperature measurements, overheat
# alerts (warning / error / critical), a location track inside the work area and an alarm for every
# critical alert.
#
# Bound: device_builder, event_builder, logger, rnd, params, geo (services/dataset_runner.py).

import time

db, eb = device_builder, event_builder
now = int(time.time() * 1000)
site_bounds = [(34.10260138703638, -84.24412965774536), (34.101837372446774, -84.24243450164795),
               (34.101517550337825, -84.24091100692749), (34.10154953265732, -84.23856675624847),
               (34.10153176473365, -84.23575580120087), (34.10409030732968, -84.23689305782318),
               (34.104996439280704, -84.23700034618376), (34.10606246444614, -84.23700034618376),
               (34.107691680235604, -84.23690915107727)]


def bounded(req, pts):
    for lat, lon in pts:
        req.coord(lat, lon)
    return req


# ---------------------------------------------------------------- customers
company = db.persist(db.new_customer_type("construction", "Construction Company")
                     .with_description("A company that manages one or more construction areas.").with_icon("building"))
sub_type = db.persist(db.new_customer_type("subcontractor", "Subcontractor")
                      .with_description("A subcontractor that works for a company.").with_icon("truck"))
acme = db.persist(db.new_customer("construction", None, "acme", "ACME Construction Company")
                  .with_description("ACME construction company manages many subcontractors and construction sites."))
for tok, name in (("subA", "Subcontractor A"), ("subB", "Subcontractor B")):
    db.persist(db.new_customer("subcontractor", "acme", tok, name)
               .with_description(name + " manages multiple construction sites."))

# ---------------------------------------------------------------- areas and zone
db.persist(db.new_area_type("construction", "Construction Area").with_description("A construction area.")
           .with_icon("truck"))
db.persist(db.new_area_type("region", "Region").with_description("Subsection of the United States.")
           .with_icon("map").with_contained_area_type("construction"))
db.persist(bounded(db.new_area("region", None, "southeast", "Southeast Region")
                   .with_description("Region including the southeastern portion of the United States."), site_bounds))
site = db.persist(bounded(db.new_area("construction", "southeast", "peachtree", "Peachtree Construction Site")
                          .with_description("A construction site with many high-value assets that should not be "
                                            "taken offsite."), site_bounds))
zone = db.persist(bounded(db.new_zone("workarea", "Work Area", "peachtree").with_border_color("#017112")
                          .with_fill_color("#1db32e").with_opacity(0.4), site_bounds))

# ---------------------------------------------------------------- device types and commands
types = {}
kinds = {"sensors": [], "personnel": [], "heavy": []}


def device_type(token, name, kind, description, **meta):
    t = db.new_device_type(token, name).with_description(description)
    for k, v in meta.items():
        t.metadata(k, v)
    types[token] = t
    kinds[kind].append(token)
    return t


def command(type_token, namespace, name, description, *params_):
    c = db.new_command(type_token, f"{type_token}-{name}", namespace, name).with_description(description)
    for pname, ptype, required in params_:
        {"String": c.with_string_parameter, "Bool": c.with_boolean_parameter}[ptype](pname, required)
    return db.persist(c)


ns = "http://sitewhere/common"
device_type("galaxytab3", "Galaxy Tab 3", "personnel", "Thin, lightweight Android tablet with a 7-inch display.",
            manufacturer="Samsung", cpu="1.2ghz", memory="1gb")
device_type("uno", "Arduino UNO", "sensors", "Microcontroller board based on the ATmega328.", manufacturer="Arduino")
device_type("mega2560", "Arduino Mega 2560", "sensors", "Microcontroller board based on the ATmega2560.",
            manufacturer="Arduino")
device_type("raspberrypi", "Raspberry Pi", "sensors", "Credit-card-sized single-board computer.",
            manufacturer="Raspberry Pi Foundation", weight="1.000", memory="2kb")
device_type("mt90", "MeiTrack MT90", "heavy", "Waterproof GPS personal tracker for assets and fleets.",
            manufacturer="MeiTrack", weight="1.000", memory="8kb")
gw = device_type("gateway", "Gateway Default", "sensors", "Sample gateway for testing nested device configurations.",
                 manufacturer="Advantech").make_composite()
schema = gw.new_schema().add_slot("Gateway Port 1", "gw1")
bus = schema.add_unit("Default Bus", "default")
bus.add_unit("PCI Bus", "pci").add_slot("PCI Device 1", "pci1").add_slot("PCI Device 2", "pci2")
bus.add_unit("Serial Ports", "serial").add_slot("COM Port 1", "com1").add_slot("COM Port 2", "com2")
schema.add_unit("High Voltage Bus 1", "hv1").add_slot("HV Slot 1", "slot1").add_slot("HV Slot 2", "slot2")
device_type("openhab", "openHAB", "sensors", "Virtual device type for testing openHAB functionality.",
            manufacturer="openHAB")
device_type("nodered", "Node-RED", "sensors", "Virtual device type for testing Node-RED functionality.",
            manufacturer="Node-RED")
device_type("laipac-S911", "S911 Bracelet Locator HC", "personnel", "Bracelet locator for patients and staff.",
            manufacturer="Laipac")
device_type("iphone6s", "Apple iPhone 6S", "personnel", "Apple phone with 3D Touch.", manufacturer="Apple")
device_type("ipad", "Apple iPad", "personnel", "12.9-inch Retina display tablet.", manufacturer="Apple")
for tok, t in types.items():
    types[tok] = db.persist(t)
    logger.info("[Create Device Type] %s", types[tok].name)

command("galaxytab3", "http://android/example", "changeBackground", "Change background color of application.",
        ("color", "String", True))
command("mega2560", "http://arduino/example", "serialPrintln", "Print a message to the serial output.",
        ("message", "String", True))
command("raspberrypi", "http://raspberrypi/example", "helloWorld", "Request a hello world response from device.",
        ("greeting", "String", True), ("loud", "Bool", True))
command("openhab", ns, "sendOnOffCommand", "Send on/off command to an openHAB item.",
        ("itemName", "String", True), ("command", "String", True))
command("openhab", ns, "sendOpenCloseCommand", "Send open/close command to an openHAB item.",
        ("itemName", "String", True), ("command", "String", True))
for tok in types:
    if tok != "galaxytab3":
        command(tok, ns, "ping", "Send a ping request to the device to verify it can be reached.")
        command(tok, ns, "testEvents", "Request that the device send a set of test events.")

# ---------------------------------------------------------------- groups
groups = {
    "heavy": db.persist(db.new_group("heavy-equipment", "Heavy Equipment Tracking").with_role("heavy-equipment-tracking")
                        .with_role("tracking").with_description("Devices tracking the location of heavy equipment.")),
    "personnel": db.persist(db.new_group("personnel", "Personnel Tracking").with_role("personnel-tracking")
                            .with_role("tracking").with_description("Devices tracking the location of people.")),
    "sensors": db.persist(db.new_group("sensors", "Sensors").with_role("monitoring").with_role("data-gathering")
                          .with_description("Sensors tracking environmental conditions.")),
}
assets = {"heavy": ["923483933-SERIAL-NUMBER-416F", "298383493-SERIAL-NUMBER-430F", "593434849-SERIAL-NUMBER-D5K2",
                    "345438345-SERIAL-NUMBER-D5K2", "847234833-SERIAL-NUMBER-320EL", "349544949-SERIAL-NUMBER-324E"],
          "personnel": ["derek.adams@sitewhere.com", "bryan.rank@sitewhere.com", "martin.weber@sitewhere.com"],
          "sensors": ["342349343-SERIAL-NUMBER-EKA4", "623947324-SERIAL-NUMBER-EKB4", "392455494-SERIAL-NUMBER-T301W",
                      "734539339-SERIAL-NUMBER-TS1", "193835744-SERIAL-NUMBER-TS1", "398434398-SERIAL-NUMBER-HS1"]}
titles = {"heavy": "Equipment Tracker", "personnel": "Personnel Tracker", "sensors": "Sensor"}


# ---------------------------------------------------------------- events
def history(assignment, start):
    """Engine-temperature / fuel measurements with overheat alerts, then a location track."""
    p = params
    t = start - int(rnd.random() * 60000)
    temp, fuel, delta = float(p["min_temp"]), 100.0, 4.0
    mx, alerts = [], []
    for _ in range(p["measurements_per_assignment"]):
        temp = round(temp + delta + (rnd.random() * 12 - 6), 2)
        if temp > p["max_temp"] or temp < p["min_temp"]:
            delta = -delta
        fuel = max(0.0, round(fuel - rnd.random() * 2, 2))
        mx.append(eb.new_measurements().measurement("fuel.level", fuel).on(t).track_state())
        mx.append(eb.new_measurements().measurement("engine.temperature", temp).on(t).track_state())
        if temp > p["warn_temp"]:
            if temp > p["critical_temp"]:
                a = eb.new_alert("engine.overheat", f"Engine shut down due to critical temperature of {temp} degrees")
                a.critical()
            elif temp > p["error_temp"]:
                a = eb.new_alert("engine.overheat", "Engine temperature is at a dangerous level.").error()
            else:
                a = eb.new_alert("engine.overheat", "Engine temperature is at top of operating range.").warning()
            alerts.append(a.on(t).track_state())
        t += int(rnd.random() * 30000)
    events = eb.for_assignment(assignment)
    events.persist_measurements(mx)
    for alert in events.persist_alerts(alerts):
        if alert.level == "Critical":             # AlertLevel is a str enum
            db.persist(db.new_device_alarm(assignment, alert.message).with_triggering_event_id(alert.id))
    # location track: a random walk that stays inside the work area
    t = start - int(rnd.random() * 60000)
    lat, lon = geo.centroid(zone.bounds)
    step = 0.0004
    dlat, dlon = (rnd.random() * 2 - 1) * step, (rnd.random() * 2 - 1) * step
    locs = []
    for _ in range(p["locations_per_assignment"]):
        for _turn in range(16):
            if geo.contains(zone.bounds, lat + dlat, lon + dlon):
                break
            dlat, dlon = -dlon, dlat                       # turn 90 degrees and try again
        if geo.contains(zone.bounds, lat + dlat, lon + dlon):
            lat, lon = lat + dlat, lon + dlon
        locs.append(eb.new_location(lat, lon).on(t).track_state())
        t += int(rnd.random() * 30000)
    events.persist_locations(locs)
    return len(mx), len(alerts), len(locs)


# ---------------------------------------------------------------- devices and assignments
members = {k: [] for k in kinds}
start = now - 2 * 3600 * 1000
for i in range(params["devices_per_site"]):
    kind = rnd.choice([k for k in kinds if kinds[k]])
    ttok = rnd.choice(kinds[kind])
    token = f"{rnd.randrange(100000)}-{ttok.upper()}-{rnd.randrange(10000000)}"
    device = db.persist(db.new_device(ttok, token).with_comment(f"{titles[kind]} based on {types[ttok].name}."))
    assignment = db.persist(db.new_assignment(device.token, "acme", "peachtree", rnd.choice(assets[kind])))
    members[kind].append(db.new_group_element(device.token))
    n_mx, n_alerts, n_locs = history(assignment, start)
    logger.info("[Create Device] %s: %d measurements, %d alerts, %d locations", device.token, n_mx, n_alerts, n_locs)
for kind, group in groups.items():
    db.persist(db.new_group(group.token, group.name), members[kind])

# ---------------------------------------------------------------- fixed demo fleet
# Deterministic tokens (<type>-NNN, commands <type>-ping...) that examples, the REST docs and the
# test-suite address directly, plus the site-boundary zone the MI355X zone-rule examples use.
demo_types = [("galaxytab", "Samsung Galaxy Tab 3 8.0", "Android tablet used by site supervisors"),
              ("meitrack", "MeiTrack GPS", "Vehicle GPS tracker")]
for tok, name, desc in demo_types:
    types[tok] = db.persist(db.new_device_type(tok, name).with_description(desc))
    command(tok, ns, "ping", "Send a ping")
    command(tok, ns, "testEvents", "Send test events")
for tok in ("galaxytab", "meitrack", "raspberrypi", "iphone6s", "openhab"):
    for suffix, desc, params_ in (("setReportingInterval", "Change reporting interval", [("interval", "Int32", True)]),
                                  ("bannerMessage", "Show a banner", [("message", "String", True)])):
        c = db.new_command(tok, f"{tok}-{suffix}", ns, suffix).with_description(desc)
        for pname, ptype, req in params_:
            {"String": c.with_string_parameter, "Int32": c.with_int32_parameter}[ptype](pname, req)
        db.persist(c)
    for code, sname, color in (("ok", "Operational", "#dcf5dc"), ("warn", "Warning", "#f5f5dc"),
                               ("err", "Error", "#f5dcdc")):
        db.persist(db.new_device_status(tok, code, sname).with_background_color(color))
db.persist(db.new_customer("subcontractor", "acme", "acme-electric", "Acme Electric"))
db.persist(bounded(db.new_zone("construction-zone", "Construction Site", "peachtree").with_border_color("#017112")
                   .with_fill_color("#1db32e").with_opacity(0.4),
                   [(34.10255918760198, -84.24389678239822), (34.101992218961306, -84.24246072769165),
                    (34.10174802166776, -84.24095541238785), (34.102315085648426, -84.2409148812294),
                    (34.102882150262455, -84.24242019653320), (34.10338396108289, -84.24368965625763)]))
supervisors = []
n = 0
for tok in ("galaxytab", "meitrack", "raspberrypi", "iphone6s", "openhab"):
    for i in range(4):
        dtok = f"{tok}-{i:03d}"
        db.persist(db.new_device(tok, dtok).with_comment(f"{tok} #{i}"))
        db.persist(db.new_assignment(dtok, "acme", "peachtree", f"asset-{n % 6}"))
        if tok == "galaxytab":
            supervisors.append(db.new_group_element(dtok, ["supervisor"]))
        n += 1
db.persist(db.new_group("supervisors", "Supervisor devices").with_role("supervisor"), supervisors)
