"""Tenant dataset templates (reference ``service-tenant-management/dockerimage/datasets/*``).

``construction`` mirrors the reference's construction-site dataset (deviceModel.groovy,
assetModel.groovy, scheduleModel.groovy): device types with commands and statuses, a customer and
area hierarchy with zones, devices assigned to assets, and schedules.  ``airtraffic`` models aircraft
trackers.  Each function is idempotent (skips if its first entity already exists).
"""
from __future__ import annotations

import random

SITE_BOUNDS = [(34.10260138703638, -84.24412965774536), (34.101837372446774, -84.24243450164795),
               (34.101517550337825, -84.24091100692749), (34.10154953265732, -84.23856675624847),
               (34.10153176473365, -84.23575580120087), (34.10409030732968, -84.23689305782318),
               (34.104996439280674, -84.23797583580017), (34.10446339273438, -84.23861503601074),
               (34.1043567821025, -84.24031019210815), (34.10418508136412, -84.24074411392212)]
ZONE_BOUNDS = [(34.10255918760198, -84.24389678239822), (34.101992218961306, -84.24246072769165),
               (34.10174802166776, -84.24095541238785), (34.102315085648426, -84.2409148812294),
               (34.102882150262455, -84.24242019653320), (34.10338396108289, -84.24368965625763)]

DEVICE_TYPES = [
    ("galaxytab", "Samsung Galaxy Tab 3 8.0", "Android tablet used by site supervisors"),
    ("meitrack", "MeiTrack GPS", "Vehicle GPS tracker"),
    ("raspberrypi", "Raspberry Pi", "Edge gateway with environmental sensors"),
    ("iphone6s", "Apple iPhone 6S", "Worker phone"),
    ("openhab", "openHAB", "Home automation bridge"),
]
COMMANDS = [("ping", "Send a ping", []), ("testEvents", "Send test events", []),
            ("setReportingInterval", "Change reporting interval", [("interval", "Int32", True)]),
            ("bannerMessage", "Show a banner", [("message", "String", True), ("color", "String", False)])]
STATUSES = [("ok", "Operational", "#dcf5dc"), ("warn", "Warning", "#f5f5dc"), ("err", "Error", "#f5dcdc")]


def bootstrap_device_model(dm, template: str, devices_per_type: int = 4, seed: int = 7):
    if template in (None, "", "empty"):
        return
    if dm.get_device_type_by_token("galaxytab" if template == "construction" else "aircraft-tracker"):
        return
    rnd = random.Random(seed)
    if template == "airtraffic":
        dm.create_device_type({"token": "aircraft-tracker", "name": "Aircraft Tracker"})
        dm.create_customer_type({"token": "airline", "name": "Airline"})
        for c in ("delta", "united", "american"):
            dm.create_customer({"token": c, "name": c.title(), "customerTypeToken": "airline"})
        dm.create_area_type({"token": "airspace", "name": "Airspace"})
        dm.create_area({"token": "atl-airspace", "name": "ATL airspace", "areaTypeToken": "airspace"})
        dm.create_zone({"token": "atl-restricted", "name": "Restricted", "areaToken": "atl-airspace",
                        "bounds": [{"latitude": a, "longitude": b} for a, b in ZONE_BOUNDS]})
        for i in range(10):
            dm.create_device({"token": f"flight-{i:03d}", "deviceTypeToken": "aircraft-tracker"})
            dm.create_device_assignment({"deviceToken": f"flight-{i:03d}",
                                         "customerToken": rnd.choice(["delta", "united", "american"]),
                                         "areaToken": "atl-airspace"})
        return
    for tok, name, desc in DEVICE_TYPES:
        dm.create_device_type({"token": tok, "name": name, "description": desc})
        for ctok, cdesc, params in COMMANDS:
            dm.create_device_command({"token": f"{tok}-{ctok}", "deviceTypeToken": tok, "namespace": "http://sitewhere/common",
                                      "name": ctok, "description": cdesc,
                                      "parameters": [{"name": p, "type": t, "required": r} for p, t, r in params]})
        for code, sname, bg in STATUSES:
            dm.create_device_status({"token": f"{tok}-{code}", "deviceTypeToken": tok, "code": code, "name": sname,
                                     "backgroundColor": bg})
    dm.create_customer_type({"token": "construction", "name": "Construction Company"})
    dm.create_customer_type({"token": "subcontractor", "name": "Subcontractor"})
    dm.create_customer({"token": "acme", "name": "Acme Construction", "customerTypeToken": "construction"})
    dm.create_customer({"token": "acme-electric", "name": "Acme Electric", "customerTypeToken": "subcontractor",
                        "parentCustomerToken": "acme"})
    dm.create_area_type({"token": "region", "name": "Region"})
    dm.create_area_type({"token": "site", "name": "Construction Site"})
    dm.create_area({"token": "southeast", "name": "Southeast", "areaTypeToken": "region"})
    dm.create_area({"token": "peachtree", "name": "Peachtree Corners Site", "areaTypeToken": "site",
                    "parentAreaToken": "southeast", "bounds": [{"latitude": a, "longitude": b} for a, b in SITE_BOUNDS]})
    dm.create_zone({"token": "construction-zone", "name": "Construction Site", "areaToken": "peachtree",
                    "bounds": [{"latitude": a, "longitude": b} for a, b in ZONE_BOUNDS],
                    "borderColor": "#017112", "fillColor": "#1db32e", "opacity": 0.4})
    dm.create_device_group({"token": "supervisors", "name": "Supervisor devices", "roles": ["supervisor"]})
    n = 0
    for tok, _, _ in DEVICE_TYPES:
        for i in range(devices_per_type):
            dtok = f"{tok}-{i:03d}"
            dm.create_device({"token": dtok, "deviceTypeToken": tok, "comments": f"{tok} #{i}"})
            dm.create_device_assignment({"deviceToken": dtok, "customerToken": "acme", "areaToken": "peachtree",
                                         "assetToken": f"asset-{n % 6}"})
            if tok == "galaxytab":
                dm.add_device_group_elements(dm.get_device_group_by_token("supervisors").id,
                                             [{"deviceToken": dtok, "roles": ["supervisor"]}])
            n += 1


def bootstrap_asset_model(am, template: str):
    if template in (None, "", "empty") or am.get_asset_type_by_token("person") is not None:
        return
    am.create_asset_type({"token": "person", "name": "Person", "assetCategory": "Person"})
    am.create_asset_type({"token": "equipment", "name": "Heavy Equipment", "assetCategory": "Hardware"})
    am.create_asset_type({"token": "tracker", "name": "Tracker", "assetCategory": "Device"})
    names = ["Derek Adams", "Bob Dole", "Jane Smith", "Excavator 12", "Bulldozer 7", "Crane 3"]
    for i, n in enumerate(names):
        am.create_asset({"token": f"asset-{i}", "name": n, "assetTypeToken": "person" if i < 3 else "equipment"})


def bootstrap_schedule_model(sm, template: str):
    if template in (None, "", "empty") or sm.get_schedule_by_token("every-hour") is not None:
        return
    sm.create_schedule({"token": "every-hour", "name": "Every hour", "triggerType": "CronTrigger",
                        "triggerConfiguration": {"cronExpression": "0 * * * *"}})
    sm.create_schedule({"token": "every-minute", "name": "Every minute", "triggerType": "SimpleTrigger",
                        "triggerConfiguration": {"repeatInterval": 60000, "repeatCount": -1}})
