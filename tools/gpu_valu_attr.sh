#!/bin/bash
# Dynamic VALU attribution for c2: one SQ_INSTS_VALU pass per library build -- the in-tree library and the
# duplication builds of tools/ab_build.sh (WCPT_DUP_PAIR / _SPHERES / _RANDDIR / _BOX run one phase's work twice
# on laundered inputs), so each build's extra VALU count is that phase's dynamic VALU. Own time limit per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-valu}
for lib in cur ${LIBS:-dpair dsph drd dbox}; do
  if [ "$lib" = "cur" ]; then unset WCPT_LIBRARY; else export WCPT_LIBRARY="wc-path-tracer_amd/variants/$lib.so"; fi
  PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" TAG=${TAG}_$lib N=1 T=120 \
    BENCH_ARGS="--config ${CFG:-c2}" bash tools/pmc_one.sh || exit 1
done
echo VALU_DONE
