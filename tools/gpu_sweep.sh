cd "${GRAFT_REPO_ROOT:?}" || exit 1; mkdir -p gpurun_out
run() {  # run one bench configuration, print a summary line; stop the sweep on any failure
  timeout -k 10 ${T:-300} python bench.py --no-cpu-baseline --host-inclusive off --ingest-leg off --mixed-leg off "$@" > gpurun_out/b.json 2> gpurun_out/b.err || { echo "FAIL $*"; tail -5 gpurun_out/b.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/b.json'));print(sys.argv[1:], d['value'], 'GiB/s', d['roofline']['kernel_ms'],'ms/launch', d['steps'], 'steps', d['config']['kernel'], d['config'].get('bytes_per_gpu',''))" "$@"
  cp gpurun_out/b.json "gpurun_out/sweep_$(echo "$*" | tr ' -' '__').json"
}
for spec in "$@"; do eval run $spec; done
echo SWEEP_DONE
