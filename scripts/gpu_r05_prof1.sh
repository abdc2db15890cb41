# round-5 profile evidence, part 1: kernel trace of the default bench, ALS / c4 / two-tower PMC passes.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python bench.py $A > gpurun_out/prof_bench.json 2> gpurun_out/prof_trace.err
ALS_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python bench.py $A $ALS_ONLY > /dev/null 2> gpurun_out/prof_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python bench.py $A $ALS_ONLY > /dev/null 2> gpurun_out/prof_write.err
C4_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_c4 -o fetchc4 -- python bench.py $A $C4_ONLY > /dev/null 2> gpurun_out/prof_fetch_c4.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_c4 -o writec4 -- python bench.py $A $C4_ONLY > /dev/null 2> gpurun_out/prof_write_c4.err
TT_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_tt -o fetchtt -- python bench.py $TT_ONLY > /dev/null 2> gpurun_out/prof_fetch_tt.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_tt -o writett -- python bench.py $TT_ONLY > /dev/null 2> gpurun_out/prof_write_tt.err
echo part1 done
