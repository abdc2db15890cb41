set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_ing_f -o f -- python scripts/ingest_probe.py > gpurun_out/pmc_ing_f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_ing_w -o w -- python scripts/ingest_probe.py > gpurun_out/pmc_ing_w.log 2>&1
python - <<'P'
import csv, glob, collections
for tag in ('f', 'w'):
    f = glob.glob('gpurun_out/pmc_ing_%s/**/*counter_collection.csv' % tag, recursive=True)[0]
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:60]
        acc[(k, r['Counter_Name'])] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
    for (k, c), v in sorted(acc.items()):
        if any(s in k for s in ('sort_', 'mark', 'codes', 'indptr', 'copy_entries', 'descent')):
            print(tag, "%-60s %-11s per-call %.3f GB" % (k, c, v / n[(k, c)] / 1e9))
P
