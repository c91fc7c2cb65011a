# Round-5 evidence, part A: PMC passes for every bench config (copied into
# profiles/ on the box so the bench lines quote them), the default bench line,
# its rocprofv3 kernel-trace summary, and smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/final_r5}
mkdir -p $O
bash scripts/gpu/pmc_all.sh "${PMC_CFGS:-c3 c3cone c4 c4csg c5}" > $O/pmc_all.log 2>&1 || { tail -5 $O/pmc_all.log; exit 1; }
for c in ${PMC_CFGS:-c3 c3cone c4 c4csg c5}; do
  cp gpurun_out/pmc_$c/pmc_$c.json profiles/pmc_$c.json && cp gpurun_out/pmc_$c/traffic.json profiles/traffic_$c.json || exit 1
done
grep -A1 "==" $O/pmc_all.log
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof -o c3 --output-format csv -- python3 bench.py --steps 30 --warmup 3 --cpu-baseline off --companion off > $O/rocprof_bench.json 2> $O/rocprof_bench.err || { tail -5 $O/rocprof_bench.err; exit 1; }
python3 scripts/trace_span.py "$(find $O/rocprof -name '*kernel_trace.csv' | head -1)" 30 $O/trace_span_c3.json
# the same run's HIP-event span (its bench line) and rocprofv3 trace span, side by side
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
line = json.loads(open(O + "/rocprof_bench.json").read().strip().splitlines()[-1])
ts = json.load(open(O + "/trace_span_c3.json"))
line["roofline"]["trace_span_ms"] = round(ts["span_ms_per_frame"], 4)
line["roofline"]["trace_span_source"] = "rocprofv3 --kernel-trace of this run (scripts/trace_span.py)"
json.dump(line, open(O + "/bench_c3_rocprof_spans.json", "w"))
print("event span", line["roofline"]["kernel_ms"], "trace span", line["roofline"]["trace_span_ms"])
PY
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
