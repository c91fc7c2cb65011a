# Repeated C3 whole-frame A/B (alternating variants, 30 steps each).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c3rep
mkdir -p $O
for i in 1 2 3; do
  for v in old s0 s1 s7; do
    lib=go-raytracer_amd/csrc/librtamd.so; unset RT_SPEC_EXTRA_FLAGS
    case $v in old) lib=build_variants/librtamd_old.so;; s1) export RT_SPEC_EXTRA_FLAGS="-DRT_QSTEAL=1";; s7) export RT_SPEC_EXTRA_FLAGS="-DRT_QSTEAL=7";; esac
    RT_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --config ${1:-c3} --steps 30 --warmup 3 --cpu-baseline off > $O/$v-$i.json 2> $O/$v-$i.err || { tail -5 $O/$v-$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v-$i.json')); print('$v', d['ms_per_step'])"
  done
done
