#!/bin/bash
# Round 4: a long random fuzz of the fused digest pairs -- 3 000 scripts from 8 threads under each
# EFES_PAIR_STAGE mode (seeds beyond the test suite's), every text and digest against the oracle.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_pair_fuzz_long}
mkdir -p "$O"
for mode in scratch cached stream; do
  EFES_PAIR_STAGE=$mode timeout -k 10 300 python3 -u - $mode > "$O/$mode.log" 2>&1 <<'PY' || { tail -30 "$O/$mode.log"; exit 1; }
import random, sys, threading, time
sys.path[:0] = [".", "tests"]
from oracle import oracle
oracle.build()
import efes_amd
from efes_amd import _lib, hashing
import test_gpu_pairs as T
mode = sys.argv[1]
base = {"scratch": 100_000, "cached": 200_000, "stream": 300_000}[mode]
gpu = dict(efes=efes_amd, hashing=hashing, lib=_lib.lib(), check=_lib.check, oracle_lib=oracle.lib())
s0 = hashing.pair_stats(); errors = []; t0 = time.time()
def worker(t):
    try:
        for k in range(t, 3000, 8):
            T._script(gpu, oracle, random.Random(base + k), 24, tag=f"{mode} seed {base + k}")
    except Exception as e:
        errors.append(repr(e)[:2000])
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[th.start() for th in ths]; [th.join() for th in ths]
s1 = hashing.pair_stats()
print(mode, {k: s1[k] - s0[k] for k in s0}, "errors", len(errors), "seconds %.1f" % (time.time() - t0))
if errors: print(errors[:3]); sys.exit(1)
PY
  tail -1 "$O/$mode.log"
done
