# Round 6: rt_render_ex band plans on one device (bench --api): equal bands
# vs decreasing bands (RT_RENDER_BAND_SHAPE=1), several band counts,
# interleaved rounds. usage: CFG=c3 bash scripts/gpu/r6_bands.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-c3}
O=${O:-gpurun_out/r6_bands_$CFG}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-"0:4" "1:3" "1:4" "1:5" "1:6" "0:3"}; do
    s=${v%%:*}; nb=${v#*:}; n=s${s}_b${nb}_r$r
    RT_RENDER_BAND_SHAPE=$s RT_RENDER_BANDS=$nb timeout -k 10 300 python3 bench.py --api --config $CFG --steps ${STEPS:-30} --warmup 3 --cpu-baseline off > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/$n.json')); p=d['seam']['last_call_parts']
print('%-12s %.4f ms/call  gpu %.3f  copy_tail %.3f  gather %.3f' % ('$n', d['ms_per_step'], p['gpu_ms'], p['copy_tail_ms'], d['seam']['gather_ms']))"
  done
done
