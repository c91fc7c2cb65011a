# Round-5 evidence, part C: the strong-scaling rehearsal (every rank's share of
# a frame at 1/2/4/8 ranks, serial and two frames in flight) for every config,
# and the brute-force C5 band (bench line, kernel stats, PMC).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/final_r5}
mkdir -p $O/strong
for c in ${INFLIGHT_CFGS:-c3 c3cone c4 c2 c4csg c5}; do
  S=20; [ $c = c5 ] && S=3; [ $c = c4csg ] && S=8
  INFLIGHT_F=${INFLIGHT_F:-1,2} timeout -k 10 400 python3 scripts/inflight_emul.py $c $S > $O/strong/inflight_$c.json 2> $O/strong/inflight_$c.err || { tail -5 $O/strong/inflight_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/strong/inflight_$c.json'))
print('$c', ' '.join('w%d: %.3f/%s' % (w, d['w%d_f2_max_ms' % w], d.get('w%d_f2_eff_max' % w)) for w in (1, 2, 4, 8)))"
done
if [ -z "$NO_BRUTE" ]; then bash scripts/gpu/brute_pmc.sh ${BRUTE_TAG:-r5final} > $O/brute.log 2>&1 || { tail -5 $O/brute.log; exit 1; }; tail -3 $O/brute.log; fi
