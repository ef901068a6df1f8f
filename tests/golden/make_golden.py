"""Generate the golden fixtures under tests/golden/ (run in the build container, committed).

Sources of truth, all independent of the C oracle and of the HIP kernels:
  * Python hashlib.sha1 / zlib.crc32 -- FIPS 180-4 SHA-1 and IEEE 802.3 CRC-32, the
    algorithms the reference vendors (sha1.go:1-9, crc32.go:1-12);
  * the reference's own known-answer test sha1file_test.go:11-12 (asserted below);
  * oracle/sha1_ref.py (pure-Python restatement of sha1.go's state machine) for the
    mid-stream MarshalText vectors, each cross-checked against hashlib for its Sum.
The synthetic byte generator is re-implemented here in numpy (not via the C oracle) so
that the C oracle's copy is checked against it too.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle.sha1_ref import Sha1Digest, crc32_marshal_text  # noqa: E402

GAMMA = np.uint64(0x9E3779B97F4A7C15)


def synthetic(n: int, seed: int) -> bytes:
    """Little-endian splitmix64 stream: z_i = mix(seed + (i+1)*gamma)."""
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, nw + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:n]


def kat():
    fox = "the quick brown fox jumps over the lazy dog\n"
    assert hashlib.sha1(fox.encode()).hexdigest() == "5d2781d78fa5a97b7bafa849fe933dfc9dc93eba"  # sha1file_test.go:11-12
    strings = ["", "hello world", "foo", "bar", "foobar", "12345", "qwerty", fox, "a" * 55, "a" * 56,
               "a" * 63, "a" * 64, "a" * 65, "b" * 119, "b" * 120, "c" * 1000]
    out = []
    for s in strings:
        b = s.encode()
        out.append({"text": s, "sha1": hashlib.sha1(b).hexdigest(), "crc32": "%08x" % zlib.crc32(b)})
    return out


EDGE_LENGTHS = [0, 1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129,
                191, 192, 255, 256, 1000, 4095, 4096, 4097, 4096 * 64 - 1, 4096 * 64, 4096 * 64 + 1,
                65536 * 3 + 7, (1 << 20) + 13]
BIG_LENGTHS = [(4 << 20) - 1, 4 << 20, (4 << 20) + 1]  # 4 MiB chunk edges (BASELINE configs)


def synthetic_vectors():
    out = []
    for i, n in enumerate(EDGE_LENGTHS + BIG_LENGTHS):
        seed = 0xEFE5 ^ (i << 32)
        b = synthetic(n, seed)
        out.append({"seed": seed, "length": n, "sha1": hashlib.sha1(b).hexdigest(),
                    "crc32": "%08x" % zlib.crc32(b)})
    return out


def state_vectors():
    """Write sequences -> MarshalText after every Write + final Sum (sha1_efes.go:25-38)."""
    rng = random.Random(1234)
    out = []
    # sha1_efes_test.go:8-29: zero-valued digest (no Reset) written "hello world".
    d = Sha1Digest(reset=False)
    d.write(b"hello world")
    out.append({"name": "zero_iv_hello_world", "reset": False, "writes": ["hello world".encode().hex()],
                "texts": [d.marshal_text()], "sum": d.sum().hex()})
    assert d.sum().hex() == "73e8730e5086d8ced928b654beeb0e5383f9be01"
    cases = [("foo_bar", [b"foo", b"bar"]), ("fox_split", [b"the quick ", b"brown fox jumps over the lazy dog\n"])]
    for k in range(24):
        total = rng.choice([1, 10, 63, 64, 65, 100, 200, 333, 1000])
        data = synthetic(total, 0x5EED + k)
        cuts = sorted(rng.sample(range(total + 1), min(rng.randint(1, 4), total + 1)))
        parts, prev = [], 0
        for c in cuts + [total]:
            parts.append(data[prev:c])
            prev = c
        cases.append((f"random_{k}", parts))
    for name, parts in cases:
        d = Sha1Digest()
        texts = []
        for p in parts:
            d.write(p)
            texts.append(d.marshal_text())
        s = d.sum().hex()
        assert s == hashlib.sha1(b"".join(parts)).hexdigest()
        out.append({"name": name, "reset": True, "writes": [p.hex() for p in parts], "texts": texts, "sum": s})
    return out


def crc_state_vectors():
    out = []
    for parts in ([b"hello world"], [b"foo", b"bar"], [synthetic(100, 7), synthetic(5, 8), b""]):
        crc, texts = 0, []
        for p in parts:
            crc = zlib.crc32(p, crc)
            texts.append(crc32_marshal_text(crc))
        out.append({"writes": [p.hex() for p in parts], "texts": texts, "sum32": crc})
    return out


def sha1file_vectors():
    """sha1file_test.go:31-35 seek/read script over the fox line."""
    content = "the quick brown fox jumps over the lazy dog\n"
    script = [[0, 9], [2, 3], [2, 7], [2, 9], [11, len(content) - 11]]
    return {"content": content, "script": script, "reads": [content[s:s + n] for s, n in script],
            "sha1": hashlib.sha1(content.encode()).hexdigest()}


def main():
    fixtures = {
        "kat.json": kat(),
        "synthetic.json": synthetic_vectors(),
        "sha1_states.json": state_vectors(),
        "crc32_states.json": crc_state_vectors(),
        "sha1file.json": sha1file_vectors(),
    }
    for name, data in fixtures.items():
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(data, f, indent=1)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
