# rocprofv3 kernel trace of the JVM-exact score + top-k probe (scripts/score_quick.py)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ps -o ps -- python scripts/score_quick.py 1024 > gpurun_out/ps.log 2>&1
python - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/ps/**/*kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last 12 dispatches = one als_score_topk call and the checks
for r in rows[-40:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f'{int(r["Start_Timestamp"])//1000 % 10**7:9d} {d:9.1f} us  grid {r.get("Grid_Size","?"):>9} {r["Kernel_Name"][:90]}')
PY
