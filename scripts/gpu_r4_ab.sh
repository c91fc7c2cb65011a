# Same-box A/B of library builds (scripts/ab.py: one process, interleaved
# rounds, specialised kernels, serial frames, outputs compared byte for byte).
# usage: bash scripts/gpu_r4_ab.sh TAG "CFGS" ROUNDS lib1 lib2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; CFGS=$2; R=$3; shift 3
O=gpurun_out/r4_$TAG
mkdir -p $O
for c in $CFGS; do
  RR=$R; [ $c = c5 ] && RR=2
  timeout -k 10 400 python3 scripts/ab.py --config $c --rounds $RR "$@" > $O/ab_$c.log 2>&1 || { tail -5 $O/ab_$c.log; exit 1; }
  echo "== $c"; cat $O/ab_$c.log
done
