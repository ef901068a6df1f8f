#!/bin/bash
# Round 4: stress of the fused digest pairs on the final tree -- the C consumer from 64 threads,
# 1 500 random pair scripts from 8 Python threads (seeds beyond the test suite's), then
# ThreadSanitizer over the consumer and the Go-surface harness (tools/gpu_r04_tsan.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_pair_stress}
mkdir -p "$O"
timeout -k 10 300 ./tests/c/efes_consumer_test 64 8 > "$O/consumer64.log" 2>&1 || { tail -20 "$O/consumer64.log"; exit 1; }
tail -3 "$O/consumer64.log"
timeout -k 10 400 python3 -u - > "$O/scripts.log" 2>&1 <<'PY' || { tail -30 "$O/scripts.log"; exit 1; }
import random, sys, threading, time
sys.path[:0] = [".", "tests"]
from oracle import oracle
oracle.build()
import efes_amd
from efes_amd import _lib, hashing
import test_gpu_pairs as T
gpu = dict(efes=efes_amd, hashing=hashing, lib=_lib.lib(), check=_lib.check, oracle_lib=oracle.lib())
s0 = hashing.pair_stats(); errors = []; t0 = time.time()
def worker(t):
    try:
        for k in range(t, 1500, 8):
            T._script(gpu, oracle, random.Random(10_000 + k), 24, tag=f"seed {10_000 + k}")
    except Exception as e:
        errors.append(repr(e)[:2000])
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[th.start() for th in ths]; [th.join() for th in ths]
s1 = hashing.pair_stats()
print({k: s1[k] - s0[k] for k in s0}, "errors", len(errors), "seconds %.1f" % (time.time() - t0))
if errors: print(errors[:3]); sys.exit(1)
print("ok")
PY
tail -2 "$O/scripts.log"
bash tools/gpu_r04_tsan.sh "${1:-r04_pair_stress}_tsan"
