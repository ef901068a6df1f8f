/*
 * efes_testing.h -- test hooks of libefeshash.so.  NOT part of the stable surface of efes_hash.h
 * (a binding such as go/hash_gpu.go never declares them): the symbols are exported so
 * the library under test is the product build, and nothing reaches them except an explicit call --
 * no environment variable or configuration switches them on.  The risk of exporting them is stated in
 * INTEGRATION.md §5.
 */
#ifndef EFES_TESTING_H
#define EFES_TESTING_H
#include <stdint.h>

#include "efes_hash.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The k-th launch from now of ctx's digest queue (k = 0: none) reports a device fault instead of
 * running, as a faulted kernel would, and the queue stays faulted: the fault-latching tests of the
 * Go surface (tests/test_gpu_boundary.py). */
int efes_debug_fault_after(efes_ctx* ctx, uint64_t k);

#ifdef __cplusplus
}
#endif
#endif /* EFES_TESTING_H */
