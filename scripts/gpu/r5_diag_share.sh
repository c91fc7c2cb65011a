# Round 5: diagnostic-build wave lifetimes and board counters of c4csg's
# rank-0 8-rank share, without sharing, with the workgroup board, with the
# device-wide board.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_diag}
mkdir -p $O
for sh in ${SHARES:-0 1 2}; do
  RT_AMD_LIB=build_variants/librtamd_phase.so RT_SPEC_EXTRA_FLAGS="-DRT_PHASE_TIMING" INFLIGHT_SHARE=$sh INFLIGHT_F=1 INFLIGHT_WORLDS=${WORLDS:-8} INFLIGHT_RANKS=0 \
    timeout -k 10 300 python3 scripts/inflight_emul.py ${CFG:-c4csg} 2 > $O/diag_share$sh.json 2> $O/diag_share$sh.err || { tail -5 $O/diag_share$sh.err; exit 1; }
  echo "== share $sh"; grep -E "share|waves|tail|passes|phase" $O/diag_share$sh.err | tail -6
done
