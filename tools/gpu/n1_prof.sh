#!/bin/bash
# rocprofv3 of the N=1 bench: kernel stats, then one PMC pass (FETCH_SIZE / WRITE_SIZE) of the
# timed K1 copy kernel (1 GB in, 1 GB out per step).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/n1prof; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/n1prof/stats -o n1 -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/n1prof/stats.log 2>&1 || exit 1
grep '^{' gpurun_out/n1prof/stats.log | cut -c1-200
find gpurun_out/n1prof/stats -name '*kernel_stats.csv' -exec cp {} gpurun_out/n1prof/n1_kernel_stats.csv \;
python3 -c "import csv; [print(r['Name'][:60], r['Calls'], r['AverageNs']) for r in list(csv.DictReader(open('gpurun_out/n1prof/n1_kernel_stats.csv')))[:3]]"
for c in FETCH_SIZE WRITE_SIZE; do   # one counter set per run (FETCH_SIZE takes 3 TCC counters)
  timeout -s KILL 90 rocprofv3 --pmc $c -f csv -d gpurun_out/n1prof/pmc_$c -o n1 -- python3 bench.py --steps 3 --warmup 1 \
    > gpurun_out/n1prof/pmc_$c.log 2>&1 || exit 1
  find gpurun_out/n1prof/pmc_$c -name '*counter_collection.csv' -exec cp {} gpurun_out/n1prof/n1_pmc_$c.csv \;
done
python3 - <<'PY'
import csv, collections
rows = [r for c in ("FETCH_SIZE", "WRITE_SIZE") for r in csv.DictReader(open(f"gpurun_out/n1prof/n1_pmc_{c}.csv"))]
agg = collections.defaultdict(list)
for r in rows:
    if "k_reduce_tile" in r["Kernel_Name"]:
        agg[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(dict)
for (d, c), v in agg.items():
    per[d][c] = sum(v)
for d, cs in sorted(per.items(), key=lambda x: int(x[0]))[-3:]:
    print("dispatch", d, {c: f"{v / 2**20:.3f} GiB" for c, v in cs.items()}, "(KB units -> GiB)")
PY
