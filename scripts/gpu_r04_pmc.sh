# round-4 evidence, part 2: the FETCH_SIZE / WRITE_SIZE passes of
# scripts/gpu_profile.sh (one counter group per run), summarised locally by
# scripts/summarize_profile.py
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --steps 3 --warmup 1"
ALS_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
C4_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
TT_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
run() { timeout -k 10 300 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/$2 -o $3 -- python bench.py $4 > /dev/null 2> gpurun_out/$2.err; echo "$2 ok"; }
run FETCH_SIZE prof_fetch fetch "$A $ALS_ONLY"
run WRITE_SIZE prof_write write "$A $ALS_ONLY"
run FETCH_SIZE prof_fetch_c4 fetchc4 "$A $C4_ONLY"
run WRITE_SIZE prof_write_c4 writec4 "$A $C4_ONLY"
run FETCH_SIZE prof_fetch_tt fetchtt "$TT_ONLY"
run WRITE_SIZE prof_write_tt writett "$TT_ONLY"
run FETCH_SIZE prof_fetch_c5 fetchc5 "$C5_ONLY"
run WRITE_SIZE prof_write_c5 writec5 "$C5_ONLY"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_ing -o fetching -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_fetch_ing.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_ing -o writeing -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_write_ing.err
echo done
