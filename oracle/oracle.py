"""ORACLE (test infrastructure only): ctypes wrapper over oracle/_build/liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product package (katacoffee_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
# the same restatement with f64 search statistics (ORA_REAL=double, ora_search.h)
LIB_F64_PATH = os.path.join(HERE, "_build", "liboracle_f64.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

_lib = None
_lib64 = None

P = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(f64=False):
    """The oracle library; f64=True: the variant with f64 search statistics."""
    global _lib, _lib64
    if f64:
        if _lib64 is None:
            if not os.path.exists(LIB_F64_PATH):
                build()
            _lib64 = _setup(ctypes.CDLL(LIB_F64_PATH))
        return _lib64
    if _lib is None:
        # ORACLE_LIB: an alternative build of the same library (tests/san sanitizer build)
        path = os.environ.get("ORACLE_LIB", LIB_PATH)
        if path == LIB_PATH and not os.path.exists(LIB_PATH):
            build()
        _lib = _setup(ctypes.CDLL(path))
    return _lib


def _setup(L):
    if True:
        L.ora_model_load.restype = P
        L.ora_sp_create.restype = P
        L.ora_sp_create.argtypes = [ctypes.c_int] * 6 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, P, ctypes.c_int,
                                                       ctypes.c_int, P, ctypes.c_int]
        L.ora_nn_forward.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P, ctypes.c_int, ctypes.c_int]
        L.ora_sp_rounds.argtypes = [P, ctypes.c_int]
        L.ora_sp_game_info.argtypes = [P, ctypes.c_int, P]
        L.ora_sp_game_nodes.argtypes = [P, ctypes.c_int, P, P, P, P, P]
        L.ora_sp_root_noised.argtypes = [P, ctypes.c_int, P]
        L.ora_sp_rows_count.argtypes = [P]
        L.ora_sp_rows.argtypes = [P, P, P, P, P, P, P]
        L.ora_sp_game_tree.argtypes = [P, ctypes.c_int, ctypes.c_int, P, P]
        L.ora_sp_free.argtypes = [P]
        L.ora_bn_merge.argtypes = [ctypes.c_int, ctypes.c_float] + [P] * 6
        L.ora_block_apply_blob.argtypes = [ctypes.c_int] * 4 + [P, ctypes.c_longlong] + [ctypes.c_int] * 3 + [P,
                                                                                                            ctypes.c_int]
        L.ora_sp_set_parallel.argtypes = [P, ctypes.c_int]
        L.ora_sp_set_netfn.argtypes = [P, P]
        L.ora_sp_set_schedule.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.ora_model_free.argtypes = [P]
        _load_tables(L)
    return L


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _load_tables(L):
    z = np.load(os.path.join(GOLDEN, "zobrist.npz"))
    t = np.load(os.path.join(GOLDEN, "tdist3.npz"))
    arrs = [np.ascontiguousarray(z[k], np.uint64) for k in ["board", "board2", "player", "size_x", "size_y"]]
    go = np.ascontiguousarray(z["game_over"], np.uint64)
    cdf = np.ascontiguousarray(t["cdf"].astype(np.float32))
    L.ora_load_tables(*[ptr(a) for a in arrs], ptr(go), ptr(cdf))
    _load_tables.keep = getattr(_load_tables, "keep", []) + arrs + [go, cdf]


NODE_DTYPE = np.dtype([
    ("visits", "<u4"), ("weightSum", "<f4"), ("weightSqSum", "<f4"), ("utilityAvg", "<f4"),
    ("utilitySqAvg", "<f4"), ("winLossAvg", "<f4"), ("nnWin", "<f4"), ("nnLoss", "<f4"),
    ("lastSvbDelta", "<f4"), ("lastSvbWeight", "<f4"), ("svbEntry", "<i4"), ("numChildren", "<u2"),
    ("nextPla", "u1"), ("flags", "u1"), ("key0", "<u8"), ("key1", "<u8"),
])
assert NODE_DTYPE.itemsize == 64


def rules_batch(X, Y, W, colors, last_cell, last_dir, pla):
    n = len(pla)
    A = X * Y
    legal = np.zeros((n, 4 * A), np.uint8)
    has = np.zeros(n, np.uint8)
    lib().ora_rules_batch(X, Y, W, n, ptr(np.ascontiguousarray(colors, np.uint8)),
                          ptr(np.ascontiguousarray(last_cell, np.int8)), ptr(np.ascontiguousarray(last_dir, np.int8)),
                          ptr(np.ascontiguousarray(pla, np.uint8)), ptr(legal), ptr(has))
    return legal, has


def play_batch(X, Y, W, colors, last_cell, last_dir, pla, move):
    n = len(pla)
    A = X * Y
    out = dict(colors=np.zeros((n, A), np.uint8), finished=np.zeros(n, np.uint8), winner=np.zeros(n, np.uint8),
               max_run=np.zeros(n, np.int32), pos_hash=np.zeros((n, 2), np.uint64), state_hash=np.zeros((n, 2), np.uint64))
    lib().ora_play_batch(X, Y, W, n, ptr(np.ascontiguousarray(colors, np.uint8)),
                         ptr(np.ascontiguousarray(last_cell, np.int8)), ptr(np.ascontiguousarray(last_dir, np.int8)),
                         ptr(np.ascontiguousarray(pla, np.uint8)), ptr(np.ascontiguousarray(move, np.int32)),
                         ptr(out["colors"]), ptr(out["finished"]), ptr(out["winner"]), ptr(out["max_run"]),
                         ptr(out["pos_hash"]), ptr(out["state_hash"]))
    return out


def encode_batch(X, Y, W, colors, hist_cell, hist_dir, pla, sym):
    n = len(pla)
    A = X * Y
    binp = np.zeros((n, 15, A), np.float32)
    glob = np.zeros(n, np.float32)
    lib().ora_encode_batch(X, Y, W, n, ptr(np.ascontiguousarray(colors, np.uint8)),
                           ptr(np.ascontiguousarray(hist_cell, np.int8)), ptr(np.ascontiguousarray(hist_dir, np.int8)),
                           ptr(np.ascontiguousarray(pla, np.uint8)), ptr(np.ascontiguousarray(sym, np.int32)),
                           ptr(binp), ptr(glob))
    return binp, glob


def fake_net(X, Y, W, binp):
    n = binp.shape[0]
    out = np.zeros((n, 4 * X * Y + 4), np.float32)
    lib().ora_fake_net(X, Y, W, n, ptr(np.ascontiguousarray(binp, np.float32)), ptr(out))
    return out


# ---- NN layer library (ora_nn.cpp), NHWC activations ----
def _f32(a):
    return np.ascontiguousarray(a, np.float32)


def conv_apply(w, x, mode=0):
    """ConvLayer: w [cout][cin][ky][kx], x [n][Y][X][cin] -> [n][Y][X][cout]."""
    cout, cin, ky, kx = w.shape
    n, Y, X, _ = x.shape
    out = np.zeros((n, Y, X, cout), np.float32)
    w, x = _f32(w), _f32(x)
    lib().ora_conv_apply(ky, kx, cin, cout, ptr(w), n, X, Y, ptr(x), ptr(out), mode)
    return out


def bn_merge(eps, mean, var, scale, bias):
    C = len(mean)
    s, b = np.zeros(C, np.float32), np.zeros(C, np.float32)
    a = [_f32(v) for v in (mean, var, scale, bias)]
    lib().ora_bn_merge(C, ctypes.c_float(eps), *[ptr(v) for v in a], ptr(s), ptr(b))
    return s, b


def bn_apply(s, b, x, mask=None, relu=False):
    n, Y, X, C = x.shape
    out = np.zeros_like(x, dtype=np.float32)
    s, b, x = _f32(s), _f32(b), _f32(x)
    m = _f32(mask) if mask is not None else None
    lib().ora_bn_apply(C, ptr(s), ptr(b), int(relu), n, X, Y, ptr(x), ptr(m) if m is not None else None, ptr(out))
    return out


def block_apply_parts(x, mask, pre, conv1, mid, conv2, gconv=None, gbn=None, linG=None, mode=0):
    """One residual block from its pieces (ResidualBlock / GlobalPoolingResidualBlock,
    eigenbackend.cpp:888-1015): pre/mid/gbn = merged (scale, bias); convs [cout][cin][ky][kx];
    linG [Cr][3Cg].  x NHWC is updated and returned."""
    n, Y, X, _ = x.shape
    x = _f32(x).copy()
    kind = 1 if gconv is not None else 0
    k1 = np.array([conv1.shape[2], conv1.shape[3], conv1.shape[1], conv1.shape[0]], np.int32)
    k2 = np.array([conv2.shape[2], conv2.shape[3], conv2.shape[1], conv2.shape[0]], np.int32)
    arrs = [_f32(pre[0]), _f32(pre[1]), _f32(conv1), _f32(mid[0]), _f32(mid[1]), _f32(conv2)]
    if kind:
        kg = np.array([gconv.shape[2], gconv.shape[3], gconv.shape[1], gconv.shape[0]], np.int32)
        g = [_f32(gconv), _f32(gbn[0]), _f32(gbn[1]), _f32(linG)]
    else:
        kg = np.zeros(4, np.int32)
        g = [np.zeros(1, np.float32)] * 4
    m = _f32(mask) if mask is not None else None
    lib().ora_block_apply_parts(kind, n, X, Y, ptr(m) if m is not None else None, ptr(x), ptr(arrs[0]), ptr(arrs[1]),
                                ptr(k1), ptr(arrs[2]), ptr(kg), ptr(g[0]), ptr(g[1]), ptr(g[2]), ptr(g[3]),
                                ptr(arrs[3]), ptr(arrs[4]), ptr(k2), ptr(arrs[5]), mode)
    return x


def block_apply_blob(kind, W, mid, Cg, blob, x, mode=0):
    """One block from its CFNN tensor sequence (kinds 0-3); x NHWC updated and returned."""
    n, Y, X, _ = x.shape
    x = _f32(x).copy()
    blob = _f32(blob)
    rc = lib().ora_block_apply_blob(kind, W, mid, Cg, ptr(blob), ctypes.c_longlong(blob.size), n, X, Y, ptr(x), mode)
    if rc != 0:
        raise ValueError("block tensors do not match kind %d at width %d" % (kind, W))
    return x


class Model:
    def __init__(self, path):
        self.h = lib().ora_model_load(path.encode())
        if not self.h:
            raise RuntimeError("oracle: cannot load model " + path)

    def forward(self, X, Y, binp, glob, mode=0, threads=1):
        n = binp.shape[0]
        A = X * Y
        pol = np.zeros((n, 4, A), np.float32)
        val = np.zeros((n, 2), np.float32)
        misc = np.zeros((n, 2), np.float32)
        lib().ora_nn_forward(self.h, X, Y, n, ptr(np.ascontiguousarray(binp, np.float32)),
                             ptr(np.ascontiguousarray(glob, np.float32)), ptr(pol), ptr(val), ptr(misc), mode, threads)
        return pol, val, misc

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_model_free(self.h)


# PlaySettings the oracle takes, in ora_sp_create order, with the benchmark-mode
# defaults of coffee_search_params_default.
PLAY_SETTINGS = {
    "cheap_search_prob": 0.0, "cheap_search_visits": 100, "cheap_search_target_weight": 0.0,
    "reduce_visits": 0, "reduce_visits_threshold": 0.9, "reduce_visits_threshold_lookback": 3,
    "reduced_visits_min": 100, "reduced_visits_weight": 0.1,
    "policy_surprise_data_weight": 0.0, "value_surprise_data_weight": 0.0,
    "init_games_with_policy": 0, "policy_init_area_prop": 0.04, "policy_init_area_temperature": 1.0,
    "early_fork_game_prob": 0.0, "early_fork_game_expected_move_prop": 0.025, "fork_game_prob": 0.0,
    "fork_game_min_choices": 3, "early_fork_game_max_choices": 12, "fork_game_max_choices": 36,
    "side_position_prob": 0.0,
    "record_tree_positions": 0, "record_tree_threshold": 0, "record_tree_target_weight": 0.0,
    "cpuct_exploration": 1.1,
}


_NETFN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


class Selfplay:
    """Round-synchronous self-play engine (select -> batched NN -> backup per round)."""

    def __init__(self, X, Y, W, games, max_visits, node_cap=2048, seed=1, slot_base=0, nn_mode=0, model=None,
                 nn_threads=1, nn_cache_log2=0, nn_batch_cap=0, f64=False, commit_interval=1, start_stagger=0,
                 **play):
        """play: PLAY_SETTINGS keywords (the device's coffee_search_params names).
        f64: search statistics in f64 (the reference's precision) instead of the
        device's f32; node dumps (nodes/game_tree) are f32-layout only.
        commit_interval / start_stagger: the device engine's round schedule
        (coffee_selfplay_config): a game whose root reached its visit limit idles
        until the next commit round ((round + 1) % commit_interval == 0, or the last
        round of a rounds() call, as kc.Selfplay.step commits); each slot idles a seeded
        number of rounds in [0, start_stagger) before its first game."""
        self.L = lib(f64)
        self.f64 = f64
        self.X, self.Y, self.W, self.games = X, Y, W, games
        self.A, self.P = X * Y, 4 * X * Y
        self.model = model
        unknown = set(play) - set(PLAY_SETTINGS)
        if unknown:
            raise TypeError("unknown play settings: %s" % sorted(unknown))
        self._play = np.array([play.get(k, d) for k, d in PLAY_SETTINGS.items()], np.float32)
        self.h = self.L.ora_sp_create(X, Y, W, games, max_visits, node_cap, seed, slot_base, nn_mode,
                                     model.h if model is not None else None, nn_threads, nn_cache_log2,
                                     ptr(self._play), nn_batch_cap)
        if not self.h:
            raise RuntimeError("oracle selfplay create failed")
        if commit_interval != 1 or start_stagger != 0:
            if self.L.ora_sp_set_schedule(self.h, int(commit_interval), int(start_stagger)) != 0:
                raise ValueError("bad schedule: commit_interval %r start_stagger %r" % (commit_interval, start_stagger))

    def rounds(self, n):
        self.L.ora_sp_rounds(self.h, n)
        if getattr(self, "_net_error", None) is not None:
            raise RuntimeError("network callback failed") from self._net_error

    def set_net(self, fn):
        """Composition tests: every later round's network batch is evaluated by
        fn(packed [n][ceil(15A/64)] u64) -> [n][P+4] f32 (coffee_nn_forward's layout),
        e.g. the device network, instead of the oracle's own forward.  None restores
        the stand-in network."""
        words = (15 * self.A + 63) // 64
        width = self.P + 4
        self._net_error = None

        def cb(n, pin, pout):
            try:
                packed = np.ctypeslib.as_array(ctypes.cast(pin, ctypes.POINTER(ctypes.c_uint64)), shape=(n, words))
                res = np.asarray(fn(packed.copy()), np.float32)
                assert res.shape == (n, width), res.shape
                np.ctypeslib.as_array(ctypes.cast(pout, ctypes.POINTER(ctypes.c_float)), shape=(n, width))[:] = res
            except BaseException as e:  # ctypes drops callback exceptions: re-raised by rounds()
                self._net_error = e

        self._cb = _NETFN(cb) if fn is not None else None
        self.L.ora_sp_set_netfn(self.h, ctypes.cast(self._cb, P) if fn is not None else None)

    def set_parallel(self, threads):
        """CPU baseline only: threads over games in select/backup (row order then
        follows thread timing; counts and per-game results are unchanged)."""
        self.L.ora_sp_set_parallel(self.h, int(threads))

    def info(self, slot):
        a = np.zeros(16, np.int64)
        self.L.ora_sp_game_info(self.h, slot, ptr(a))
        keys = ["phase", "rootK", "nodeCount", "rootIdx", "turn", "pla", "gameNum", "playouts", "nnEvals",
                "movesMade", "gamesFinished", "rngCtr", "leafKind", "rootVisits", "lastCell", "lastDir"]
        return dict(zip(keys, a.tolist()))

    def nodes(self, slot, cap=4096):
        if self.f64:
            raise ValueError("raw node records have the f32 layout only")
        nodes = np.zeros(cap, NODE_DTYPE)
        ec = np.zeros(cap * self.P, np.uint32)
        ev = np.zeros(cap * self.P, np.uint32)
        em = np.zeros(cap * self.P, np.uint16)
        pol = np.zeros(cap * self.P, np.float32)
        n = self.L.ora_sp_game_nodes(self.h, slot, ptr(nodes), ptr(ec), ptr(ev), ptr(em), ptr(pol))
        P = self.P
        return dict(nodes=nodes[:n], edge_child=ec[:n * P].reshape(n, P), edge_visits=ev[:n * P].reshape(n, P),
                    edge_move=em[:n * P].reshape(n, P), policy=pol[:n * P].reshape(n, P))

    def root_noised(self, slot):
        out = np.zeros(self.P, np.float32)
        self.L.ora_sp_root_noised(self.h, slot, ptr(out))
        return out

    def rows(self):
        n = self.L.ora_sp_rows_count(self.h)
        A, P = self.A, self.P
        pb = (A + 7) // 8
        r = dict(binaryInputNCHWPacked=np.zeros((n, 15, pb), np.uint8), globalInputNC=np.zeros((n, 1), np.float32),
                 policyTargetsNCMove=np.zeros((n, 2, P), np.int16), globalTargetsNC=np.zeros((n, 64), np.float32),
                 valueTargetsNCHW=np.zeros((n, 5, self.Y, self.X), np.int8), meta=np.zeros((n, 4), np.int32))
        self.L.ora_sp_rows(self.h, ptr(r["binaryInputNCHWPacked"]), ptr(r["globalInputNC"]),
                          ptr(r["policyTargetsNCMove"]), ptr(r["globalTargetsNC"]), ptr(r["valueTargetsNCHW"]),
                          ptr(r["meta"]))
        return r

    def game_tree(self, slot, max_nodes=4096):
        nodes = np.zeros((max_nodes, 24), np.uint32)
        edges = np.zeros((max_nodes, self.P, 3), np.uint32)
        n = self.L.ora_sp_game_tree(self.h, slot, max_nodes, ptr(nodes), ptr(edges))
        return nodes[:n], edges[:n]

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ora_sp_free(self.h)
