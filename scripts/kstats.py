"""Summarise a rocprofv3 kernel_stats.csv by category (per step)."""
import csv
import re
import sys

CATS = [
    ("conv", r"igemm|conv|gtcx|Conv|xdl|naive_conv|transpose_NHWC|implicit"),
    ("miopen_misc", r"SubTensorOp|MIOpen"),
    ("tbamd_bn", r"tbamd::bn_"),
    ("tbamd_other", r"tbamd::"),
    ("gemm", r"Cijk|gemm|Gemm|hipblaslt"),
    ("pool", r"pool"),
    ("copy_cast", r"copy_kernel|bfloat16tofloat32|float32tobfloat16"),
    ("elementwise", r"elementwise|Functor|clamp"),
    ("reduce", r"reduce"),
]


def main(path, steps=1):
    rows = list(csv.DictReader(open(path)))
    agg = {}
    tot = 0.0
    for r in rows:
        t = float(r["TotalDurationNs"]) / 1e6
        tot += t
        for c, pat in CATS:
            if re.search(pat, r["Name"]):
                break
        else:
            c = "other"
        agg[c] = agg.get(c, 0.0) + t
    print(f"total {tot/steps:.2f} ms/step ({steps} steps)")
    for c, t in sorted(agg.items(), key=lambda x: -x[1]):
        print(f"  {c:14s} {t/steps:8.2f} ms/step  {100*t/tot:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
