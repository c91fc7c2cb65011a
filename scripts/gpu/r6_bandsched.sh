# Round 6: the seam's per-band schedule (pick_schedule sees a band's pixels)
# vs serial samples for every band (RT_PIXEL_QUADS=0), C3 bench --api;
# interleaved rounds; then the bench's own rt_render leg at the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_bandsched}
mkdir -p $O
for r in 1 2; do
  for v in auto serial; do
    n=${v}_r$r
    if [ $v = serial ]; then export RT_PIXEL_QUADS=0; else unset RT_PIXEL_QUADS; fi
    timeout -k 10 300 python3 bench.py --api --config c3 --steps 30 --warmup 3 --cpu-baseline off > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$n.json')); s=d['seam']; p=s['last_call_parts']
print('%-10s %.4f ms/call gpu %.3f tail %.3f  first %.1f ms, %d calls to specialise' % ('$n', d['ms_per_step'], p['gpu_ms'], p['copy_tail_ms'], s['first_call_ms'], s['calls_until_specialised']))"
  done
done
unset RT_PIXEL_QUADS
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_default.json')); a=d['render_api']
print('bench', d['ms_per_step'], 'render_api steady', a['steady_ms'], a['parts_ms'], 'calls', a['calls'])"
