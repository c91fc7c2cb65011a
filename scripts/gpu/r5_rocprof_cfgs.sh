# Round 5: rocprofv3 kernel-trace summaries of the other bench configs' default
# lines (C4, c4csg, C5), next to the C3 one from final_a.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/final_r5/rocprof_cfgs}
mkdir -p $O
for c in c4 c4csg c5; do
  s=20; [ $c = c5 ] && s=3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$c -o $c --output-format csv -- python3 bench.py --config $c --steps $s --warmup 2 --cpu-baseline off --companion off > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 scripts/trace_span.py "$(find $O/$c -name '*kernel_trace.csv' | head -1)" $s $O/trace_span_$c.json > /dev/null
  python3 -c "import json; d=json.load(open('$O/$c.json')); t=json.load(open('$O/trace_span_$c.json')); print('$c', d['ms_per_step'], 'event span', d['roofline']['kernel_ms'], 'trace span', round(t['span_ms_per_frame'], 4))"
done
