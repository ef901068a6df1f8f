# configs[3]'s planned parts after efes_hash_host has run in the same process (round 3: the
# per-call CU-masked copy streams of the host leg left the mixed leg at 1.39 s per step).
cd "${GRAFT_REPO_ROOT:?}" || exit 1; O=gpurun_out/stream_check; mkdir -p $O
B="--no-cpu-baseline --sha1-leg off --uploads-leg off --receiver-leg off --drain-leg off --concurrency-leg off --span-leg off --ingest-leg off"
run() { local tag=$1; shift; timeout -k 10 300 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));m=d.get('mixed_config');h=d.get('host_inclusive');print(sys.argv[2],'main',d['value'],'host',h and h['value'],'mixed',m and (m['value'],m['roofline']['kernel_ms']))" $O/$tag.json $tag; }
run plain env EFES_PART_STREAMS=plain python bench.py $B --host-inclusive on --mixed-leg on
run masked python bench.py $B --host-inclusive on --mixed-leg on
run main_masked python bench.py $B --host-inclusive off --workload mixed --steps 2 --warmup 1
run full python bench.py --no-cpu-baseline
