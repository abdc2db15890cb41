set -e
python -c "import __graft_entry__ as g; g.build()"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --no-cpu-baseline --steps 3 > gpurun_out/bench1_prof.json 2> gpurun_out/bench1_prof.err
