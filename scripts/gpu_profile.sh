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
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- python bench.py $A --no-ingest --score-users 0 --hybrid-users 0 > /dev/null 2> gpurun_out/prof_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- python bench.py $A --no-ingest --score-users 0 --hybrid-users 0 > /dev/null 2> gpurun_out/prof_write.err
python scripts/summarize_profile.py gpurun_out > gpurun_out/prof_summary.json
cat gpurun_out/prof_summary.json
