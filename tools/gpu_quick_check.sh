# The -m gpu suite and one default-flags bench line on the current tree (quick evidence after a change).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; O=gpurun_out/quick; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --ingest-leg off --mixed-leg off"
timeout -k 10 300 python bench.py $B --host-inclusive on > $O/host.json 2> $O/host.err || { tail -5 $O/host.err; exit 1; }
python -c "import json;d=json.load(open('$O/host.json'));print('headline',d['value'],'host_inclusive',d['host_inclusive']['value'],d['host_inclusive']['digests_match_device_path'])"
