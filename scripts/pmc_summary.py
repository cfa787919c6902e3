"""Summarise rocprofv3 --pmc CSVs (gpurun_out/rNN/pmc_*) per kernel over the last steady-state steps.

Usage: python scripts/pmc_summary.py gpurun_out/r37 [n_last_dispatches]
Derived (gfx950, 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs):
  cycles      = GRBM_GUI_ACTIVE / 8
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * 1024)
  mfma_tflops ~ SQ_VALU_MFMA_BUSY_CYCLES * 1024 FLOP (bf16 16x16x32: 16 cycles, 16384 FLOP) / kernel time
  lds_conf    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_GB      = (2 * FETCH_SIZE + WRITE_SIZE) KiB (FETCH_SIZE reads 1/2 of wide streams on gfx950)
"""
import collections
import csv
import sys


def load(path, last):
    rows = list(csv.DictReader(open(path)))
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    keep = set(ids[-last:])
    per = collections.defaultdict(dict)
    name, dur = {}, {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d not in keep:
            continue
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per, name, dur


def short(n):
    n = n.replace("tbamd::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def main():
    root = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 527
    sq, nm, du = load(f"{root}/pmc_sq/run_counter_collection.csv", last)
    fe, nmf, _ = load(f"{root}/pmc_fetch/run_counter_collection.csv", last)
    wr, nmw, _ = load(f"{root}/pmc_write/run_counter_collection.csv", last)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d, c in sq.items():
        k = short(nm[d])
        a = agg[k]
        a["calls"] += 1
        a["t"] += du[d]
        for key, v in c.items():
            a[key] += v
    for src, names in ((fe, nmf), (wr, nmw)):
        for d, c in src.items():
            for key, v in c.items():
                if key != "GRBM_GUI_ACTIVE":
                    agg[short(names[d])][key] += v
    tot_t = sum(a["t"] for a in agg.values())
    print(f"last {last} dispatches of each pass; kernel time under PMC serialisation {tot_t*1e3:.2f} ms")
    print(f"{'kernel':70s} {'calls':>5s} {'ms':>7s} {'mfma%':>6s} {'TF/s':>6s} {'ldsconf%':>8s} {'HBM GB':>7s} {'TB/s':>5s}")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["t"])[:30]:
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        util = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024) * 100 if cyc else 0
        tf = a["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / a["t"] / 1e12 if a["t"] else 0
        lds = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"] * 100 if a["SQ_LDS_IDX_ACTIVE"] else 0
        gb = (2 * a.get("FETCH_SIZE", 0) + a.get("WRITE_SIZE", 0)) * 1024 / 1e9
        bw = gb / a["t"] / 1e3 if a["t"] else 0
        print(f"{k:70s} {int(a['calls']):5d} {a['t']*1e3:7.3f} {util:6.1f} {tf:6.0f} {lds:8.2f} {gb:7.3f} {bw:5.2f}")


if __name__ == "__main__":
    main()
