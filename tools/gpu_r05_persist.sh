set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r05_ac; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit 1; }
for pp in 1 2 3; do run blk_p$pp 300 python3 -u tools/block_balance.py --config c3 --ns 4,8 --skip-full --wf-pipes $pp; done
for f in 0 1; do run full_c3_persist$f 300 python3 -u bench.py --config c3 --no-cpu-baseline --steps 30 --wf-persist $f; done
run full_c2ref 300 python3 -u tools/block_balance.py --config ref --ns 8 --skip-full --kernel 2 --wf-persist 1
echo SESSION_DONE
