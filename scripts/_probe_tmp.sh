set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dot.py -k "filter or dot_topk or prune or hybrid or recommender" > gpurun_out/filter_tests.log 2>&1 || { tail -30 gpurun_out/filter_tests.log; exit 1; }
tail -1 gpurun_out/filter_tests.log
C5_ONLY="--no-ingest --score-users 0 --hybrid-users 0 --c4-items 0 --tt-steps 0 --api-reps 0 --rank256-epochs 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 python bench.py $C5_ONLY > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
python - <<'P'
import json
d = json.loads(open('gpurun_out/c5_bench.json').read().strip().splitlines()[-1])
def find(o, k):
    if isinstance(o, dict):
        if k in o: return o[k]
        for v in o.values():
            r = find(v, k)
            if r is not None: return r
c5 = find(d, 'hybrid_top5_c5')
print({k: c5[k] for k in ('ms_per_batch', 'eager_ms_per_batch', 'graph_ms_per_batch', 'launch')})
r = c5['roofline']
print('survivors', r.get('survivors_per_user'), 'fallback', r.get('fallback_taken'))
for st in r['stages']: print(round(st['avg_launch_ms'], 4), st['kernel'][:60] if 'kernel' in st else st.get('name', '')[:60])
print(r.get('batch_view'))
P
bash scripts/prof_c5.sh > /dev/null 2>&1
grep -E "hp_|dot_res|topk|hyb_" gpurun_out/prof_c5_gaps.txt | tail -9
