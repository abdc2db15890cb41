# rocprofv3 evidence for the bench's dominant kernel (run via gpurun):
#   1) kernel trace + stats of the default bench workload
#   2) PMC FETCH_SIZE pass, 3) PMC WRITE_SIZE pass (separate passes: the TCC
#      slots cannot hold both; MI355X_MICROARCH.md §rocprofv3 PMC slots)
# then summarises into gpurun_out/prof_summary.json (copied to profiles/).
set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="--no-cpu-baseline --steps 3 --warmup 1 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python bench.py $A > gpurun_out/prof_bench.json 2> gpurun_out/prof_trace.err
ALS_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python bench.py $A $ALS_ONLY > /dev/null 2> gpurun_out/prof_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python bench.py $A $ALS_ONLY > /dev/null 2> gpurun_out/prof_write.err
# c4 two-tower scoring (dot_res_kernel): its own FETCH_SIZE pass
C4_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c5-users 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_c4 -o fetchc4 -- python bench.py $A $C4_ONLY > /dev/null 2> gpurun_out/prof_fetch_c4.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_c4 -o writec4 -- python bench.py $A $C4_ONLY > /dev/null 2> gpurun_out/prof_write_c4.err
# two-tower train step: the grouped whole-table Adam sweep (adam_sparse_group4_kernel), FETCH and WRITE passes
TT_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --c5-users 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_tt -o fetchtt -- python bench.py $TT_ONLY > /dev/null 2> gpurun_out/prof_fetch_tt.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_tt -o writett -- python bench.py $TT_ONLY > /dev/null 2> gpurun_out/prof_write_tt.err
# c5 pruned hybrid (hyb_scores_kernel HS_PRUNE, dot_res_kernel FILTER, hp_*): FETCH and WRITE passes
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_c5 -o fetchc5 -- python bench.py $C5_ONLY > /dev/null 2> gpurun_out/prof_fetch_c5.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_c5 -o writec5 -- python bench.py $C5_ONLY > /dev/null 2> gpurun_out/prof_write_c5.err
# ingest (encode + CSR/CSC radix build): FETCH and WRITE passes of the probe
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_ing -o fetching -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_fetch_ing.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_ing -o writeing -- python scripts/ingest_probe.py > /dev/null 2> gpurun_out/prof_write_ing.err
# rank-256 ALS half-sweeps (als_half_sweep_wide_kernel): kernel trace of the probe
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide -o wide -- python scripts/wide_quick.py 256 300000 100000 > gpurun_out/prof_wide.log 2>&1
python scripts/summarize_profile.py gpurun_out > gpurun_out/prof_summary.json
cat gpurun_out/prof_summary.json
