# Air-traffic dataset: asset management initializer (reference
# datasets/airtraffic/scripts/asset-management/content/initializer/assetModel.groovy): employees,
# flight-management units and aircraft types, with one asset per tracked aircraft.

ab = asset_builder
for tok, name, category in (("employee", "SiteWhere Employee", "Person"), ("FMZ2000", "FMZ 2000", "Device"),
                            ("A330-200", "Airbus A330-200", "Hardware"), ("A330-300", "Airbus A330-300", "Hardware"),
                            ("BOEING-717", "Boeing 717", "Hardware"), ("BOEING-737", "Boeing 737-700", "Hardware")):
    ab.persist(ab.new_asset_type(tok, name, category))
for tok, name in (("derek.adams@sitewhere.com", "Derek Adams"), ("bryan.rank@sitewhere.com", "Bryan Rank"),
                  ("martin.weber@sitewhere.com", "Martin Weber")):
    ab.persist(ab.new_asset("employee", tok, name))
for i in range(params["flights"]):
    typ = ("A330-200", "A330-300", "BOEING-717", "BOEING-737")[i % 4]
    ab.persist(ab.new_asset(typ, f"aircraft-{i:03d}", f"{typ} #{i}"))
