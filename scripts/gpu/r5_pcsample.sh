# Round 5: instruction-level PC sampling of the C3 bench kernel (rocprofv3 beta).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_pcs}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/list.txt 2>&1; echo "list rc=$?"
grep -i -A12 "pc sampling\|pc_sampling\|PC Sampling" $O/list.txt | head -40
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-host_trap} --pc-sampling-unit ${PCS_UNIT:-time} --pc-sampling-interval ${PCS_INT:-1000} \
  -d $O/run -o pcs --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off --companion off --inflight 1 > $O/bench.json 2> $O/bench.err
echo "pcs rc=$?"; tail -3 $O/bench.err; find $O/run -type f | head; du -sh $O/run
