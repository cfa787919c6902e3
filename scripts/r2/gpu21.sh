# E7 AdaIN b32@256 native vs stock; route tables for adain/online/dcgan; ResNet-50 colsum sweep
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_21
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
TBAMD_TUNE_LOG=1 timeout -k 10 700 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native --save-routes $O/routes_adain.json > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-220 $O/adain_native.json
timeout -k 10 400 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode stock > $O/adain_stock.json 2> $O/adain_stock.err
chk $? adain_stock; cut -c1-220 $O/adain_stock.json
for CS in 64,64 16,256 32,128; do
TBAMD_COLSUM=$CS timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_$CS.json 2> $O/bench_$CS.err
chk $? bench_$CS; cut -c1-120 $O/bench_$CS.json
done
