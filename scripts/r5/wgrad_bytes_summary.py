"""Summarise gpurun_out/r5_40: per ResNet-50 weight-gradient shape, the bytes of its third run
(wgrad kernel + split reduce) against the operand minimum.  python scripts/r5/wgrad_bytes_summary.py DIR"""
import collections
import csv
import re
import sys


def passes(path, counter):
    rows = list(csv.DictReader(open(path)))
    per = collections.OrderedDict()
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        if d not in per:
            per[d] = [r["Kernel_Name"], 0.0, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3]
        per[d][1] += float(r["Counter_Value"])
    return [v for _, v in sorted(per.items())]


def main(d):
    shapes = [l.strip() for l in open(f"{d}/pf.log") if l.startswith("shape ")]
    f = [x for x in passes(f"{d}/pf/run_counter_collection.csv", "FETCH_SIZE") if re.search("wgrad", x[0])]
    w = [x for x in passes(f"{d}/pw/run_counter_collection.csv", "WRITE_SIZE") if re.search("wgrad", x[0])]
    # per shape: 3 runs, each 1 or 2 dispatches (wgrad kernel [+ wgrad_reduce_k])
    i = j = 0
    tot_min = tot_got = 0.0
    print(f"{'shape':64s} {'min MB':>7s} {'kernel MB':>9s} {'reduce MB':>9s} {'x min':>6s} {'us':>7s}")
    for s in shapes:
        mn = float(re.search(r"min_operand_MB=([\d.]+)", s).group(1))
        runs = []
        for _ in range(3):
            k = [f[i]]
            kw = [w[j]]
            i += 1
            j += 1
            if i < len(f) and "wgrad_reduce" in f[i][0]:
                k.append(f[i])
                kw.append(w[j])
                i += 1
                j += 1
            runs.append((k, kw))
        k, kw = runs[-1]
        # FETCH_SIZE / WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half of wide streams (scripts/pmc_summary.py)
        kern = (2 * k[0][1] + kw[0][1]) / 1024
        red = (2 * k[1][1] + kw[1][1]) / 1024 if len(k) > 1 else 0.0
        us = sum(x[2] for x in k)
        tot_min += mn
        tot_got += kern + red
        print(f"{s[6:70]:64s} {mn:7.1f} {kern:9.1f} {red:9.1f} {(kern + red) / mn:6.2f} {us:7.1f}")
    print(f"total: minimum {tot_min:.0f} MB, measured {tot_got:.0f} MB ({tot_got / tot_min:.2f}x)")


if __name__ == "__main__":
    main(sys.argv[1])
