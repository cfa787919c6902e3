"""Merge conv autotune tables (ops/conv.py save_routes output) into the shipped gfx950 table:
python scripts/merge_routes.py routes_a.json [routes_b.json ...]  (later files win)."""
import json
import os
import sys

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "torchbooster_amd", "ops",
                       "conv_routes_gfx950.json")


def main(paths):
    table = {}
    for p in [SHIPPED] + list(paths):
        for key, name in json.load(open(p)).get("routes", []):
            table[json.dumps(key)] = name
    rows = [f"[{k}, {json.dumps(v)}]" for k, v in sorted(table.items())]
    with open(SHIPPED, "w") as f:
        f.write('{\n"device": "gfx950",\n"routes": [\n' + ",\n".join(rows) + "\n]}\n")
    print(f"{len(rows)} routes -> {SHIPPED}")


if __name__ == "__main__":
    main(sys.argv[1:])
