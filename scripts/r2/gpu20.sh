# generic conv microbench on the DCGAN edge shape + NST shapes; kernel split under rocprofv3
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_20
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
BF16_ONLY=1 timeout -k 10 200 python scripts/r2/conv_any_bench.py dcgan_d_in,style_in,style_out,adain_out,style_down1,style_up1 > $O/bench.jsonl 2> $O/bench.err
chk $? bench; cat $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp && cd $R
BF16_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ca -- python scripts/r2/conv_any_bench.py dcgan_d_in > $O/prof.log 2>&1
chk $? prof
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r2_20/prof/ca_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>4}  {r["Name"][:150]}')
PY
