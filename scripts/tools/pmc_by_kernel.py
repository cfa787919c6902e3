"""Per-kernel-name means of rocprofv3 --pmc counters (all dispatches), derived MFMA util and
LDS conflict rate.  Usage: python pmc_by_kernel.py counter_collection.csv [more.csv ...]"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
dur = collections.defaultdict(dict)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        d = (path, r["Dispatch_Id"])
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[n].add(d)
        dur[n][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
for n, c in acc.items():
    k = len(cnt[n])
    m = {a: v / k for a, v in c.items()}
    ms = sum(dur[n].values()) / max(1, len(dur[n]))
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    out = [f"{n:60s} n={k:3d} ms={ms:.4f}"]
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        out.append(f"mfma={100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.1f}%")
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if key in m:
                out.append(f"{key[3:]}={m[key] / wc:.2f}")
    if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        out.append(f"ldsconf={100 * m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.1f}%")
    for key in ("SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_WAIT_INST_LDS"):
        if key in m:
            out.append(f"{key[3:]}={m[key]:.3g}")
    if cyc:
        out.append(f"clk={cyc / (ms * 1e3):.0f}MHz")
    print(" ".join(out))
