# Local: copy a final rehearsal's results (gpurun_out/$SRC) into profiles/ (PMC raw CSVs
# + regenerated summaries, bench line, rocprofv3 summary + trace span, sweep, strong, GPU log).
# usage: SRC=final_r5 DST=profiles/r05/final bash scripts/collect_final.sh
set -e
cd "$(dirname "$0")/.."
R=${R:-r05}
SRC=gpurun_out/${SRC:-final_r5}
DST=${DST:-profiles/$R/final}
mkdir -p $DST/sweep $DST/strong profiles/$R/pmc_csv
for c in c3 c3cone c4 c4csg c5; do
  for p in p1 p2 p3 p4; do cp gpurun_out/pmc_$c/$p/${p}_counter_collection.csv profiles/$R/pmc_csv/${c}_${p}_counter_collection.csv; done
  cp gpurun_out/pmc_$c/cal_f/cal_f_counter_collection.csv profiles/$R/pmc_csv/${c}_calf_counter_collection.csv
  cp gpurun_out/pmc_$c/cal_w/cal_w_counter_collection.csv profiles/$R/pmc_csv/${c}_calw_counter_collection.csv
  python3 scripts/pmc_roofline.py "profiles/$R/pmc_csv/${c}_p[12]_*.csv" profiles/pmc_$c.json rt_render > /dev/null
  python3 scripts/pmc_traffic.py "profiles/$R/pmc_csv/${c}_p[34]_*.csv" profiles/traffic_$c.json "profiles/$R/pmc_csv/${c}_cal[fw]_*.csv" > /dev/null
  mkdir -p $DST/pmc_$c && cp gpurun_out/pmc_$c/summary.txt $DST/pmc_$c/
done
cp $SRC/bench_default.json $DST/bench_c3.json
cp $SRC/rocprof_bench.json $SRC/smoke.log $DST/
cp $SRC/bench_c3_rocprof_spans.json $DST/ 2>/dev/null || true
cp $SRC/rocprof/c3_kernel_stats.csv $DST/kernel_stats_c3.csv
cp $SRC/rocprof/c3_kernel_trace.csv $DST/kernel_trace_c3.csv
python3 scripts/trace_span.py $DST/kernel_trace_c3.csv 30 $DST/trace_span_c3.json > /dev/null
cp $SRC/sweep/*.json $DST/sweep/ 2>/dev/null || true
cp $SRC/strong/*.json $DST/strong/ 2>/dev/null || true
cp $SRC/pytest_gpu.log $DST/ 2>/dev/null || true
echo collected into $DST
# brute-force C5 band (part C: scripts/gpu/brute_pmc.sh r5final)
B=gpurun_out/brute_${BRUTE_TAG:-r5final}
if [ -d $B ]; then
  mkdir -p $DST/brute
  for p in p1 p2; do cp $B/$p/${p}_counter_collection.csv profiles/$R/pmc_csv/c5bf_${p}_counter_collection.csv; done
  python3 scripts/pmc_roofline.py "profiles/$R/pmc_csv/c5bf_p[12]_*.csv" profiles/pmc_c5_bf_rows2048-2304.json rt_render > /dev/null
  cp $B/bench.json $B/summary.txt $B/kernel_stats.csv $DST/brute/ 2>/dev/null || true
  cp $B/phase.err $DST/brute/ 2>/dev/null || true
fi
cp $SRC/strong/*.err $DST/strong/ 2>/dev/null || true
cp $SRC/pmc_all.log $DST/ 2>/dev/null || true
