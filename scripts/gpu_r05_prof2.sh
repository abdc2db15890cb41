# round-5 profile evidence, part 2: c5, c2 exact hybrid, ingest PMC passes; rank-256 trace.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_c5 -o fetchc5 -- python bench.py $C5_ONLY > /dev/null 2> gpurun_out/prof_fetch_c5.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_c5 -o writec5 -- python bench.py $C5_ONLY > /dev/null 2> gpurun_out/prof_write_c5.err
HX_ONLY="--no-ingest --score-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_hx -o fetchhx -- python bench.py $HX_ONLY > /dev/null 2> gpurun_out/prof_fetch_hx.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_hx -o writehx -- python bench.py $HX_ONLY > /dev/null 2> gpurun_out/prof_write_hx.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_ing -o fetching -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_fetch_ing.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_ing -o writeing -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_write_ing.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o wide -- python scripts/wide_quick.py 256 300000 100000 > gpurun_out/prof_wide.log 2>&1
echo part2 done
