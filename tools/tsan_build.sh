#!/bin/bash
# ThreadSanitizer build of the HOST code (the reference runs `go test -race`): the
# library's host side (dispatcher, queue, uploads, streaming digests) instrumented with
# -fsanitize=thread via -Xarch_host (device code untouched), and the uploads harness and the C
# consumer of the digest surface and the Go-surface harness linked against it.  Outputs (git-ignored):
# efes_amd/lib/tsan/libefeshash.so, tools/bench_uploads_tsan, tests/c/efes_consumer_test_tsan,
# tools/bench_go_surface_tsan.
set -e
cd "$(dirname "$0")/.."
mkdir -p efes_amd/lib/tsan
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Xarch_host -fsanitize=thread -I include \
  -o efes_amd/lib/tsan/libefeshash.so efes_amd/csrc/efes_kernels.hip efes_amd/csrc/efes_crc_span.hip efes_amd/csrc/efes_api.cpp \
  efes_amd/csrc/efes_ingest.cpp efes_amd/csrc/efes_queue.cpp efes_amd/csrc/efes_stream.cpp efes_amd/csrc/efes_plan.cpp
$HIPCC -O1 -g -std=c++17 -fsanitize=thread -I include tools/bench_uploads.cpp -o tools/bench_uploads_tsan \
  -L efes_amd/lib/tsan -lefeshash -Wl,-rpath,'$ORIGIN/../efes_amd/lib/tsan' -pthread
/opt/rocm/lib/llvm/bin/clang -O1 -g -std=c11 -fsanitize=thread -pthread tests/c/efes_consumer_test.c \
  -o tests/c/efes_consumer_test_tsan -L efes_amd/lib/tsan -lefeshash -L oracle -loracle \
  -Wl,-rpath,'$ORIGIN/../../efes_amd/lib/tsan' -Wl,-rpath,'$ORIGIN/../../oracle'
$HIPCC -O1 -g -std=c++17 -fsanitize=thread -I include tools/bench_go_surface.cpp -o tools/bench_go_surface_tsan \
  -L efes_amd/lib/tsan -lefeshash -Wl,-rpath,'$ORIGIN/../efes_amd/lib/tsan' -pthread
