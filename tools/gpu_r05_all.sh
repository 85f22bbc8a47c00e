#!/bin/bash
# Round 5 closing session in one call: GPU tests + smoke + the counter passes (tools/gpu_r05_final.sh), the summaries
# copied into this box's profiles/ so the bench lines price their rooflines from this build's own profiles, then the
# bench lines, the block balance, the c3 block kernel trace and the group / RCCL rehearsals (tools/gpu_r05_session.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05_all}
TAG=$TAG/final bash tools/gpu_r05_final.sh || exit 1
S=gpurun_out/$TAG/final/summaries
cp $S/sq_*.json $S/valu_mix_*.json $S/pmc_traffic_*.json profiles/ || exit 1
TAG=$TAG/session TESTS=0 BENCH=1 BENCH_ALL=1 C4=1 BALANCE=1 KTRACE=1 GROUP=${GROUP:-1} bash tools/gpu_r05_session.sh || exit 1
echo ALL_SESSIONS_DONE
