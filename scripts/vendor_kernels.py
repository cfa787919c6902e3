"""List the vendor-library compute kernels in rocprofv3 kernel traces.

Usage: python scripts/vendor_kernels.py trace1.csv [trace2.csv ...]
Vendor = MIOpen convolutions (igemm / naive_conv / ck:: / MIOpen* solvers), hipBLASLt /
rocBLAS GEMMs (Cijk_*), and ATen compute kernels (at::native ...) -- the latter listed
separately since most are tiny elementwise glue.  Exit status 0 always; prints a table."""
import collections
import csv
import re
import sys

VENDOR = re.compile(r"igemm|naive_conv|ck::|^Cijk_|MIOpen|miopen|gridwise|conv_fwd_nhwc|_bwd_data|_wrw_", re.I)


def main():
    for path in sys.argv[1:]:
        rows = list(csv.DictReader(open(path)))
        tot = collections.Counter()
        dur = collections.Counter()
        for r in rows:
            n = r["Kernel_Name"]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            if VENDOR.search(n):
                k = "VENDOR " + n.split("(")[0][:90]
            elif "at::native" in n:
                k = "aten   " + re.sub(r"<.*", "", n.split("(")[0].replace("void at::native::", ""))[:60]
            else:
                k = "native"
            tot[k] += 1
            dur[k] += d
        all_us = sum(dur.values())
        print(f"== {path}: {len(rows)} dispatches, {all_us / 1e3:.2f} ms kernel time")
        for k, c in sorted(tot.items(), key=lambda kv: -dur[kv[0]]):
            print(f"  {dur[k] / 1e3:8.3f} ms {100 * dur[k] / max(all_us, 1e-9):5.1f} % {c:6d}  {k}")


if __name__ == "__main__":
    main()
