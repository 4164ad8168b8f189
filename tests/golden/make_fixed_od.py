"""Extract the reference's fixed-OD fixtures (all seven MA_ver1/*.xlsx: fixedDrone.xlsx,
fixedDrone_2_drone.xlsx, fixedDrone_3drones.xlsx, fixedDrone_3dronesV2.xlsx, fixedDrone_3drones_2.xlsx,
fixedDrone_5_adj.xlsx, reward_test.xlsx) into tests/golden/fixed_od.json.  The xlsx files are read as zipped sheet XML (data only; nothing
from the reference is executed).  Parsing follows reset_world_fixedOD (ATT/env:513-614): numeric gx/gy
is one goal; string cells "x1; x2" / "y1; y2" hold two waypoints, read exactly as the reference does
(x from the first token of each cell, y from the second, ATT/env:225-227 pattern)."""
import json
import os
import re
import sys
import zipfile

REF = "/root/reference/MA_ver1"
FILES = ("fixedDrone.xlsx", "fixedDrone_2_drone.xlsx", "fixedDrone_3drones.xlsx", "fixedDrone_3dronesV2.xlsx",
         "fixedDrone_3drones_2.xlsx", "fixedDrone_5_adj.xlsx", "reward_test.xlsx")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixed_od.json")


def read_rows(path):
    z = zipfile.ZipFile(path)
    sst = re.findall(r"<t[^>]*>([^<]*)</t>", z.read("xl/sharedStrings.xml").decode())
    xml = z.read("xl/worksheets/sheet1.xml").decode()
    rows = []
    for row in re.findall(r"<row [^>]*>(.*?)</row>", xml):
        vals = []
        for t, v in re.findall(r'<c r="[A-Z]+\d+"(?: s="\d+")?( t="s")?[^>]*><v>([^<]*)</v></c>', row):
            vals.append(sst[int(v)] if t else float(v))
        rows.append(vals)
    return rows[0], rows[1:]


def parse(rows):
    out = []
    for r in rows:
        start = [r[0], r[1]]
        if isinstance(r[2], str):
            xs = [int(c.split("; ")[0]) for c in r[2:4]]
            ys = [int(c.split("; ")[1]) for c in r[2:4]]
            goals = [[float(xs[0]), float(xs[1])], [float(ys[0]), float(ys[1])]]
        else:
            goals = [[r[2], r[3]]]
        out.append({"start": start, "goals": goals})
    return out


def main():
    data = {}
    for name in FILES:
        header, rows = read_rows(os.path.join(REF, name))
        data[name] = {"header": header, "agents": parse(rows)}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=1)
    print(json.dumps(data))


if __name__ == "__main__":
    sys.exit(main())
