#!/bin/bash
# AddressSanitizer build of the HOST code: the library's host side (digest layer, queue, dispatcher)
# instrumented with -fsanitize=address via -Xarch_host (device code untouched), and the lifecycle
# test of INTEGRATION.md §2's Go binding linked against it (tests/c/efes_lifecycle_test.c, run by
# tests/test_gpu_lifecycle.py).  Outputs (git-ignored): efes_amd/lib/asan/libefeshash.so,
# tests/c/efes_lifecycle_test_asan.
set -e
cd "$(dirname "$0")/.."
mkdir -p efes_amd/lib/asan
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CLANG=${CLANG:-/opt/rocm/lib/llvm/bin/clang}
$HIPCC --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer -std=c++17 -fPIC -shared -Xarch_host -fsanitize=address \
  -I include -o efes_amd/lib/asan/libefeshash.so efes_amd/csrc/efes_kernels.hip efes_amd/csrc/efes_crc_span.hip \
  efes_amd/csrc/efes_api.cpp efes_amd/csrc/efes_ingest.cpp efes_amd/csrc/efes_queue.cpp efes_amd/csrc/efes_stream.cpp \
  efes_amd/csrc/efes_plan.cpp
$CLANG -O1 -g -fno-omit-frame-pointer -std=c11 -fno-gpu-sanitize -Xarch_host -fsanitize=address -pthread \
  tests/c/efes_lifecycle_test.c -o tests/c/efes_lifecycle_test_asan -L efes_amd/lib/asan -lefeshash -L oracle -loracle \
  -Wl,-rpath,'$ORIGIN/../../efes_amd/lib/asan' -Wl,-rpath,'$ORIGIN/../../oracle'
