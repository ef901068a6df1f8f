# Round 5: the -m gpu suite on the current tree, then the clock meter on the bench's own legs
# (headline DEEP, configs[4] WIDE ingest) with a GRBM_GUI_ACTIVE pass over the same ingest run.
cd "${GRAFT_REPO_ROOT:?}" || exit 1; O=gpurun_out/${1:-r05_check}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --host-inclusive off --sha1-leg off --uploads-leg off --go-surface-leg off --latency-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --mixed-leg off"
timeout -k 10 300 python bench.py $B > $O/bench_clock.json 2> $O/bench_clock.err || { tail -5 $O/bench_clock.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_clock.json'))
print('headline', d['value'], d['clock'], d['binding_roofline'])
i=d['ingest_config']; print('ingest', i['value'], i['clock'], i['binding_roofline'])"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc_clock -o run -- python3 bench.py $B > $O/pmc_clock.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc_clock.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, json, collections
O = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{O}/pmc_clock/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        k = r["Kernel_Name"].split("(")[0]
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if ns > 1e6:
            agg[k].append(float(r["Counter_Value"]) / 8 / ns)
for k, v in agg.items():
    print(f"GRBM clock {k}: n={len(v)} median {sorted(v)[len(v)//2]*1000:.1f} MHz min {min(v)*1000:.1f} max {max(v)*1000:.1f}")
d = json.loads(open(f"{O}/pmc_clock.log").read().strip().splitlines()[-1])
print("same run's meter: headline", d["clock"], "ingest", d["ingest_config"]["clock"])
PY
