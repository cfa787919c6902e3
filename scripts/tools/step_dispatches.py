"""Dispatches of the last training step in a rocprofv3 CSV (kernel trace or counter collection):
the dispatches after the second-to-last fused-AdamW launch (one per step), printed as a count."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
disp = {}
for r in rows:
    disp[int(r["Dispatch_Id"])] = r["Kernel_Name"]
ids = sorted(disp)
steps = [i for i in ids if "adamw_mt_k<1" in disp[i]]
print(len([i for i in ids if i > steps[-2]]) if len(steps) >= 2 else len(ids) // 5)
