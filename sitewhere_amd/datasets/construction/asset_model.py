# Construction-site dataset: asset management initializer (reference
# datasets/construction/scripts/asset-management/content/initializer/assetModel.groovy): employees,
# Ekahau tags and sensors, Caterpillar heavy equipment -- the assets the device model assigns
# trackers to -- plus the fixed demo assets asset-0..asset-5.

ab = asset_builder
asset_types = [("employee", "SiteWhere Employee", "Person", None),
               ("ekahau-a4", "Ekahau A4 Tag", "Device", "Ekahau"), ("ekahau-b4", "Ekahau B4 Tag", "Device", "Ekahau"),
               ("ekahau-T301W", "Ekahau T301W Wearable Tag", "Device", "Ekahau"),
               ("ekahau-TS1", "Ekahau Wireless TS1 Temperature Sensor", "Device", "Ekahau"),
               ("ekahau-TS2", "Ekahau Wireless TS2 Temperature Sensor", "Device", "Ekahau"),
               ("ekahau-HS1", "Ekahau HS1 Humidity Sensor", "Device", "Ekahau"),
               ("cat416f", "Caterpillar 416F Backhoe Loader", "Hardware", "Caterpillar"),
               ("cat430f", "Caterpillar 430F Backhoe Loader", "Hardware", "Caterpillar"),
               ("catD5K2", "Caterpillar D5K2 Dozer", "Hardware", "Caterpillar"),
               ("cat320EL", "Caterpillar 320E L Excavator", "Hardware", "Caterpillar"),
               ("cat324E", "Caterpillar 324E Excavator", "Hardware", "Caterpillar"),
               ("person", "Person", "Person", None), ("equipment", "Heavy Equipment", "Hardware", None)]
for tok, name, category, maker in asset_types:
    t = ab.new_asset_type(tok, name, category)
    if maker:
        t.metadata("manufacturer", maker)
    ab.persist(t)

people = [("derek.adams@sitewhere.com", "Derek Adams", "derek", "dev"),
          ("bryan.rank@sitewhere.com", "Bryan Rank", "bryan", "sales"),
          ("martin.weber@sitewhere.com", "Martin Weber", "martin", "dev")]
for tok, name, user, role in people:
    ab.persist(ab.new_asset("employee", tok, name).metadata("username", user).metadata("role", role))
for tok, typ, name in (("342349343-SERIAL-NUMBER-EKA4", "ekahau-a4", "Ekahau A4 Tag 1"),
                       ("623947324-SERIAL-NUMBER-EKB4", "ekahau-b4", "Ekahau B4 Tag 1"),
                       ("392455494-SERIAL-NUMBER-T301W", "ekahau-T301W", "Ekahau T301W Tag 1"),
                       ("734539339-SERIAL-NUMBER-TS1", "ekahau-TS1", "Ekahau TS1 Sensor 1"),
                       ("193835744-SERIAL-NUMBER-TS1", "ekahau-TS1", "Ekahau TS1 Sensor 2"),
                       ("398434398-SERIAL-NUMBER-HS1", "ekahau-HS1", "Ekahau HS1 Sensor 1"),
                       ("923483933-SERIAL-NUMBER-416F", "cat416f", "Caterpillar 416F 1"),
                       ("298383493-SERIAL-NUMBER-430F", "cat430f", "Caterpillar 430F 1"),
                       ("593434849-SERIAL-NUMBER-D5K2", "catD5K2", "Caterpillar D5K2 1"),
                       ("345438345-SERIAL-NUMBER-D5K2", "catD5K2", "Caterpillar D5K2 2"),
                       ("847234833-SERIAL-NUMBER-320EL", "cat320EL", "Caterpillar 320E L 1"),
                       ("349544949-SERIAL-NUMBER-324E", "cat324E", "Caterpillar 324E 1")):
    ab.persist(ab.new_asset(typ, tok, name))
for i, name in enumerate(["Derek Adams", "Bob Dole", "Jane Smith", "Excavator 12", "Bulldozer 7", "Crane 3"]):
    ab.persist(ab.new_asset("person" if i < 3 else "equipment", f"asset-{i}", name))
