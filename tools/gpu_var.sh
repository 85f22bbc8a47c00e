set -u
for w in 3 100 400; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --warmup $w 2>&1 | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' | tr '\n' ' ' || exit 1; echo " warmup=$w"
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline --warmup 400 --steps 200 2>&1 | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' | tr '\n' ' ' || exit 1; echo " warmup=400 steps=200"
echo ALL_DONE
