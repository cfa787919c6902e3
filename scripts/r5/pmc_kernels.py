"""Per-kernel PMC table of a rocprofv3 --pmc counter_collection CSV (any program): calls, ms,
MFMA busy %, and the wave-cycle split (SQ_WAIT_ANY = parked on waitcnt / barrier, SQ_WAIT_INST_ANY =
issue stalls, SQ_ACTIVE_INST_ANY), LDS bank conflicts.  Usage: pmc_kernels.py <csv> [name-filter]"""
import collections
import csv
import re
import sys


def main(path, filt=""):
    per = collections.defaultdict(dict)
    name, dur = {}, {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
        dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d, c in per.items():
        n = name[d]
        if filt and not re.search(filt, n):
            continue
        k = n.replace("tbamd::", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        a = agg[k]
        a["calls"] += 1
        a["t"] += dur[d]
        for key, v in c.items():
            a[key] += v
    print(f"{'kernel':90s} {'n':>3s} {'ms/call':>8s} {'mfma%':>6s} {'wait%':>6s} {'stall%':>6s} {'act%':>6s} {'ldsc%':>6s}")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["t"]):
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
        mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024) * 100 if cyc else 0
        wc = a.get("SQ_WAVE_CYCLES", 0) or 1
        w = a.get("SQ_WAIT_ANY", 0) / wc * 100
        s = a.get("SQ_WAIT_INST_ANY", 0) / wc * 100
        ac = a.get("SQ_ACTIVE_INST_ANY", 0) / wc * 100
        lds = a.get("SQ_LDS_BANK_CONFLICT", 0) / a["SQ_LDS_IDX_ACTIVE"] * 100 if a.get("SQ_LDS_IDX_ACTIVE") else 0
        print(f"{k:90s} {int(a['calls']):3d} {a['t'] / a['calls'] * 1e3:8.4f} {mf:6.1f} {w:6.1f} {s:6.1f} {ac:6.1f} {lds:6.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
