# Round 6: the Render() seam timed (bench.py --api) on C3 / c4csg, one GPU and
# virtual device slots; the default bench line for regressions.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_api}
mkdir -p $O
for c in c3 c4csg; do
  timeout -k 10 300 python3 bench.py --api --config $c --steps 20 --warmup 3 --cpu-baseline off > $O/api_$c.json 2> $O/api_$c.err || { tail -5 $O/api_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/api_$c.json')); s=d['seam']; print('$c', 'ms/step', d['ms_per_step'], 'first', s['first_call_ms'], s['first_call_parts'], 'switch', s['calls_until_specialised'], 'dev', s['device_kernel_ms'], 'gather', s['gather_ms'])"
done
for devs in 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do
  timeout -k 10 300 python3 bench.py --api --api-devices $devs --config c3 --steps 20 --warmup 3 --cpu-baseline off > $O/api_c3_$devs.json 2> $O/api_c3_$devs.err || { tail -5 $O/api_c3_$devs.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/api_c3_$devs.json')); s=d['seam']; print('c3 slots $devs', 'ms/step', d['ms_per_step'], 'dev', s['device_kernel_ms'], 'gather', s['gather_ms'])"
done
timeout -k 10 600 python3 bench.py --cpu-baseline off > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('bench', d['ms_per_step'], d['value'], d['config']['tile_order_ms'], d['config']['spec_compile_ms'], d['render_api']['first_call_ms'], d['render_api']['steady_ms'], d['render_api']['first_call_parts'])"
