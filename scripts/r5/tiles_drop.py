"""Write the shipped GEMM tile table minus the ViT-B/16 b128 rows (25216 token rows), so a tuning
run re-times them with every candidate (hipBLASLt included): tiles_drop.py OUT"""
import json
import os
import sys

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                       "torchbooster_amd", "ops", "gemm_tiles_gfx950.json")
rows = json.load(open(SHIPPED))["tiles"]
keep = [r for r in rows if 25216 not in r[0][1:4] or (len(sys.argv) > 2 and r[0][0] != sys.argv[2])]
json.dump({"device": "gfx950", "tiles": keep}, open(sys.argv[1], "w"))
print(f"{len(rows) - len(keep)} rows dropped, {len(keep)} kept")
