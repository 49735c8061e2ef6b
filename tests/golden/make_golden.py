"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE implementation.

Runs oracle/_ref/refgen (built by oracle/ref/build_ref.sh from the reference's own
cpp/core + cpp/game sources) and converts its binary output into small .npz files.
Only needs to run in the build container (where /root/reference exists); the
resulting .npz files are committed and are what the tests read.

    python tests/golden/make_golden.py
"""
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFGEN = os.path.join(REPO, "oracle", "_ref", "refgen")

RULES_CONFIGS = [
    # (x, y, winLen, games, seed)
    (5, 5, 4, 400, 1),
    (7, 7, 5, 150, 2),
    (9, 9, 5, 80, 3),
    (6, 4, 3, 120, 4),
    (10, 10, 5, 25, 5),
]


def run(*args):
    subprocess.run([REFGEN, *map(str, args)], check=True)


def parse_rules(path):
    with open(path, "rb") as f:
        data = f.read()
    X, Y, W, ngames = struct.unpack_from("<4i", data, 0)
    A = X * Y
    off = 16
    recs = {k: [] for k in ["hdr", "colors", "legal", "hash_before", "after", "hash_after"]}
    while off < len(data):
        recs["hdr"].append(struct.unpack_from("<8i", data, off)); off += 32
        recs["colors"].append(np.frombuffer(data, np.uint8, A, off)); off += A
        recs["legal"].append(np.frombuffer(data, np.uint8, 4 * A, off)); off += 4 * A
        recs["hash_before"].append(np.frombuffer(data, np.uint64, 2, off)); off += 16
        recs["after"].append(struct.unpack_from("<3i", data, off)); off += 12
        recs["hash_after"].append(np.frombuffer(data, np.uint64, 6, off)); off += 48
    hdr = np.array(recs["hdr"], np.int32)
    return dict(
        dims=np.array([X, Y, W, ngames], np.int32),
        game=hdr[:, 0], turn=hdr[:, 1], pla=hdr[:, 2], last_x=hdr[:, 3], last_y=hdr[:, 4],
        last_dir=hdr[:, 5], has_legal=hdr[:, 6], move_pos=hdr[:, 7],
        colors=np.stack(recs["colors"]), legal=np.stack(recs["legal"]),
        hash_before=np.stack(recs["hash_before"]),
        after=np.array(recs["after"], np.int32), hash_after=np.stack(recs["hash_after"]),
    )


def main():
    if not os.path.exists(REFGEN):
        subprocess.run([os.path.join(REPO, "oracle", "ref", "build_ref.sh")], check=True)
    tmp = "/tmp/katacoffee_golden"
    os.makedirs(tmp, exist_ok=True)
    for (x, y, w, n, seed) in RULES_CONFIGS:
        out = os.path.join(tmp, f"rules_{x}x{y}_{w}.bin")
        run("rules", x, y, w, n, seed, out)
        np.savez_compressed(os.path.join(HERE, f"rules_{x}x{y}_{w}.npz"), **parse_rules(out))
    # Zobrist tables (board.cpp:134-178)
    out = os.path.join(tmp, "zobrist.bin")
    run("zobrist", out)
    with open(out, "rb") as f:
        data = f.read()
    max_len, arr = struct.unpack_from("<2i", data, 0)
    off = 8
    def take(n):
        nonlocal off
        a = np.frombuffer(data, np.uint64, 2 * n, off).reshape(n, 2); off += 16 * n
        return a
    np.savez_compressed(
        os.path.join(HERE, "zobrist.npz"), max_len=np.int32(max_len), arr_size=np.int32(arr),
        player=take(4), size_x=take(max_len + 1), size_y=take(max_len + 1),
        board=take(arr * 4).reshape(arr, 4, 2), board2=take(arr * 4).reshape(arr, 4, 2),
        game_over=take(1)[0])
    # Rand KATs (rand.cpp)
    out = os.path.join(tmp, "rand.bin")
    run("rand", out)
    with open(out, "rb") as f:
        data = f.read()
    (n,) = struct.unpack_from("<i", data, 0)
    off = 4
    kat = {}
    for i in range(n):
        (ln,) = struct.unpack_from("<i", data, off); off += 4
        seed = data[off:off + ln].decode(); off += ln
        u32 = np.frombuffer(data, np.uint32, 64, off); off += 256
        u64 = np.frombuffer(data, np.uint64, 64, off); off += 512
        dbl = np.frombuffer(data, np.float64, 64, off); off += 512
        gau = np.frombuffer(data, np.float64, 64, off); off += 512
        gam = np.frombuffer(data, np.float64, 80, off).reshape(5, 16); off += 640
        kat[f"seed{i}"] = np.frombuffer(seed.encode(), np.uint8)
        kat[f"u32_{i}"] = u32; kat[f"u64_{i}"] = u64; kat[f"dbl_{i}"] = dbl
        kat[f"gauss_{i}"] = gau; kat[f"gamma_{i}"] = gam
    kat["n"] = np.int32(n)
    kat["gamma_shapes"] = np.array([0.05, 0.3, 1.0, 2.5, 10.0])
    np.savez_compressed(os.path.join(HERE, "rand_kat.npz"), **kat)
    # t-distribution CDF table (search.cpp:111-116)
    out = os.path.join(tmp, "tdist.bin")
    run("tdist", out)
    with open(out, "rb") as f:
        data = f.read()
    (size,) = struct.unpack_from("<i", data, 0)
    minz, maxz = struct.unpack_from("<2d", data, 4)
    tab = np.frombuffer(data, np.float64, 2 * size, 20).reshape(size, 2)
    np.savez_compressed(os.path.join(HERE, "tdist3.npz"), minz=minz, maxz=maxz, cdf=tab[:, 0], pdf=tab[:, 1])
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
