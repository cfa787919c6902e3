"""Merge GEMM tile decisions (ops/gemm.py save_tiles output, e.g. from runs with
TBAMD_GEMM_SAVE=path) into the shipped gfx950 table; later files win:
python scripts/merge_tiles.py tiles_a.json [tiles_b.json ...]"""
import json
import os
import sys

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "torchbooster_amd", "ops",
                       "gemm_tiles_gfx950.json")


def main(paths):
    table = {}
    for p in ([SHIPPED] if os.path.exists(SHIPPED) else []) + list(paths):
        for key, cfg in json.load(open(p)).get("tiles", []):
            table[json.dumps(key)] = cfg
    rows = [f"[{k}, {json.dumps(v)}]" for k, v in sorted(table.items())]
    with open(SHIPPED, "w") as f:
        f.write('{\n"device": "gfx950",\n"tiles": [\n' + ",\n".join(rows) + "\n]}\n")
    print(f"{len(rows)} tiles -> {SHIPPED}")


if __name__ == "__main__":
    main(sys.argv[1:])
