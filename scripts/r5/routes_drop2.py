"""Write the shipped conv route table minus the batch-256 1x1 stride-1 forward / input-gradient rows
of stages 2-4 (spatial <= 28), so a tuning run re-times them with the single-stage big-tile
candidates (big128x256s1 / big256x128s1): routes_drop2.py OUT"""
import json
import os
import sys

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "torchbooster_amd", "ops", "conv_routes_gfx950.json")
rows = json.load(open(SHIPPED))["routes"]


def drop(k):
    return (k[0] in ("fwd", "dgrad") and isinstance(k[1], list) and k[1][:1] == [256] and k[2][2:] == [1, 1]
            and k[3] == 1 and k[1][2] <= 28)


keep = [r for r in rows if not drop(r[0])]
json.dump({"device": "gfx950", "routes": keep}, open(sys.argv[1], "w"))
print(f"{len(rows) - len(keep)} rows dropped, {len(keep)} kept")
