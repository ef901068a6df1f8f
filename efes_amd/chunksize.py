"""ChunkSize (chunksize.go): the K/M/G byte-size type that sets efes' PATCH chunk size.

The client sends an upload as PATCH requests of ChunkSize bytes (write.go:126, default 50M in
config.go:80, CLI default 1M in main.go:31), and every PATCH is one resumed hash call; the
benchmark's mixed workload draws its sizes from these values.
Semantics follow chunksize.go exactly: Set (17-54) parses an optional K/M/G suffix with
strconv.ParseInt (base 10, optional sign, int64 range) and multiplies with int64 wrap-around;
String (56-78) picks the largest of G/M/K that divides the value.
"""
from __future__ import annotations

K, M, G = 1024, 1024 * 1024, 1024 * 1024 * 1024
_I64 = 1 << 64


def _wrap64(v: int) -> int:
    v %= _I64
    return v - _I64 if v >= 1 << 63 else v


def _parse_int(s: str) -> int:
    """strconv.ParseInt(s, 10, 64): [+-]digits, no spaces/underscores, range-checked."""
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        raise ValueError(f'strconv.ParseInt: parsing "{s}": invalid syntax')
    v = int(s)
    if not -(1 << 63) <= v < 1 << 63:
        raise ValueError(f'strconv.ParseInt: parsing "{s}": value out of range')
    return v


def parse(value: str) -> int:
    """ChunkSize.Set (chunksize.go:17-54).  An empty string panics in Go (index out of range)."""
    if value == "":
        raise IndexError("index out of range [-1]")
    mult = {"K": K, "M": M, "G": G}.get(value[-1])
    if mult is None:
        return _parse_int(value)
    return _wrap64(_parse_int(value[:-1]) * mult)


def format(c: int) -> str:  # noqa: A001 - mirrors ChunkSize.String (chunksize.go:56-78)
    if c == 0:
        return "0"
    i, postfix = c, ""
    if _go_mod(i, G) == 0:
        i, postfix = _go_div(i, G), "G"
    elif _go_mod(i, M) == 0:
        i, postfix = _go_div(i, M), "M"
    elif _go_mod(i, K) == 0:
        i, postfix = _go_div(i, K), "K"
    return str(i) + postfix


def _go_div(a: int, b: int) -> int:  # Go integer division truncates toward zero
    q = abs(a) // b
    return q if a >= 0 else -q


def _go_mod(a: int, b: int) -> int:
    return a - _go_div(a, b) * b


# The eleven ChunkSize values of the mixed benchmark (64K .. 64M).
MIXED_CLASSES = [parse(f"{64 << k}K") if k < 4 else parse(f"{1 << (k - 4)}M") for k in range(11)]


def mixed_geometry(n: int, pool_bytes: int, seed: int = 7):
    """BASELINE configs[3]'s batch: n chunk sizes drawn uniformly from MIXED_CLASSES, longest first
    (equal lengths per WIDE wave, LPT tail), each at a seeded 256-B aligned offset of a pool of
    `pool_bytes` (chunks alias the pool: 752 GiB of chunks over 200 GiB at n = 65 536).  One function
    for bench.py's mixed leg and its full-size parity test, so both hash the same geometry.
    Returns (sizes, offsets) as uint64 arrays."""
    import numpy as np

    rng = np.random.default_rng(seed)
    sizes = np.asarray(MIXED_CLASSES, dtype=np.uint64)[rng.integers(0, len(MIXED_CLASSES), n)]
    sizes = np.sort(sizes)[::-1].copy()
    offs = (rng.integers(0, (pool_bytes - sizes.astype(np.int64)) // 256 + 1) * 256).astype(np.uint64)
    return sizes, offs
