"""Write the shipped conv route table minus the batch-256 forward / stride-1 input-gradient rows
(so a tuning run re-times them, now with the big-tile candidates): routes_drop.py OUT"""
import json
import os
import sys

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "torchbooster_amd", "ops", "conv_routes_gfx950.json")
rows = json.load(open(SHIPPED))["routes"]
keep = [r for r in rows if not (r[0][0] in ("fwd", "dgrad") and isinstance(r[0][1], list) and r[0][1][:1] == [256]
                                 and r[0][3] == 1)]
json.dump({"device": "gfx950", "routes": keep}, open(sys.argv[1], "w"))
print(f"{len(rows) - len(keep)} rows dropped, {len(keep)} kept")
