"""efes_amd: MI355X-native content hashing (SHA-1 + CRC-32/IEEE) for putdotio/efes.

The product is libefeshash.so (C ABI: include/efes_hash.h; HIP kernels for gfx950 in
efes_amd/csrc/).  This package is its Python host layer:
  efes_amd.hashing -- the reference's digest surface (sha1digest, crc32digest, Sha1File,
                      fileinfo Digest/FileInfo), GPU-backed;
  efes_amd.batch   -- device-resident batches of independent jobs (the hot path), fixed-shape
                      or planned (efes_plan_batch: grouped-DEEP parts beside WIDE).
"""
from ._lib import (EFES_ERR_ARG, EFES_ERR_DEVICE_FAULT, EFES_ERR_HIP, EFES_ERR_INVALID_DIGEST,  # noqa: F401
                   EFES_ERR_NO_DEVICE, EFES_ERR_NOMEM, EFES_ERR_STATE, EFES_JOB_FINALIZE, EFES_JOB_INIT, EFES_OK, MODE_AUTO,
                   MODE_DEEP, MODE_GROUP, MODE_WIDE, EfesError, lib)

__version__ = "0.1.0"
