"""MI355X Coffee self-play engine — Python host mirror of the C ABI.

The product is ``libkatacoffee.so`` (HIP kernels for gfx950 behind the C ABI in
``include/katacoffee.h``).  This module only binds it with ctypes and moves
arrays through torch device tensors; it has no compute path of its own and
raises if the library is missing or no GPU is present.

Reference interfaces mirrored here (same argument meaning and error behaviour):
  rules/encoder  Board::isLegal board.cpp:185-227, NNInputs::fillRowV1 nninputs.cpp:508-657
  network        NeuralNet::getOutput nninterface.h:31-171
  self-play      `katago selfplay` command/selfplay.cpp:44-72, Play::runGame play.cpp:1146-1701
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libkatacoffee.so")
CSRC = os.path.join(HERE, "csrc")

NUM_SPATIAL = 15
COFFEE_OK = 0
# network precision / path (include/katacoffee.h COFFEE_NN_*)
PRECISIONS = {"default": 0, "accurate": 1, "fast-layered": 2, "corrected": 3, "accurate-nb2": 4, "fast": 5}
PRECISION_NAMES = {v: k for k, v in PRECISIONS.items()}

_lib = None

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_u64 = ctypes.c_uint64


class CoffeeError(RuntimeError):
    pass


class SearchParams(ctypes.Structure):
    _fields_ = [
        ("max_visits", ctypes.c_int32),
        ("cpuct_exploration", ctypes.c_float), ("cpuct_exploration_log", ctypes.c_float),
        ("cpuct_exploration_base", ctypes.c_float),
        ("fpu_reduction_max", ctypes.c_float), ("root_fpu_reduction_max", ctypes.c_float),
        ("fpu_loss_prop", ctypes.c_float), ("root_fpu_loss_prop", ctypes.c_float),
        ("fpu_parent_weight_by_visited_policy", ctypes.c_int32),
        ("fpu_parent_weight_by_visited_policy_pow", ctypes.c_float),
        ("value_weight_exponent", ctypes.c_float),
        ("root_noise_enabled", ctypes.c_int32),
        ("root_dirichlet_noise_total_concentration", ctypes.c_float),
        ("root_dirichlet_noise_weight", ctypes.c_float),
        ("root_policy_temperature", ctypes.c_float), ("root_policy_temperature_early", ctypes.c_float),
        ("root_desired_per_child_visits_coeff", ctypes.c_float),
        ("root_num_symmetries_to_sample", ctypes.c_int32),
        ("chosen_move_temperature", ctypes.c_float), ("chosen_move_temperature_early", ctypes.c_float),
        ("chosen_move_temperature_halflife", ctypes.c_float),
        ("chosen_move_subtract", ctypes.c_float), ("chosen_move_prune", ctypes.c_float),
        ("use_lcb_for_selection", ctypes.c_int32),
        ("lcb_stdevs", ctypes.c_float), ("min_visit_prop_for_lcb", ctypes.c_float),
        ("subtree_value_bias_factor", ctypes.c_float), ("subtree_value_bias_weight_exponent", ctypes.c_float),
        ("subtree_value_bias_free_prop", ctypes.c_float),
        ("use_graph_search", ctypes.c_int32),
        ("cheap_search_prob", ctypes.c_float), ("cheap_search_visits", ctypes.c_int32),
        ("cheap_search_target_weight", ctypes.c_float), ("reduce_visits", ctypes.c_int32),
        ("reduce_visits_threshold", ctypes.c_float), ("reduce_visits_threshold_lookback", ctypes.c_int32),
        ("reduced_visits_min", ctypes.c_int32), ("reduced_visits_weight", ctypes.c_float),
        ("policy_surprise_data_weight", ctypes.c_float), ("value_surprise_data_weight", ctypes.c_float),
        ("init_games_with_policy", ctypes.c_int32), ("policy_init_area_prop", ctypes.c_float),
        ("policy_init_area_temperature", ctypes.c_float),
        ("early_fork_game_prob", ctypes.c_float), ("early_fork_game_expected_move_prop", ctypes.c_float),
        ("fork_game_prob", ctypes.c_float), ("fork_game_min_choices", ctypes.c_int32),
        ("early_fork_game_max_choices", ctypes.c_int32), ("fork_game_max_choices", ctypes.c_int32),
        ("side_position_prob", ctypes.c_float),
        ("record_tree_positions", ctypes.c_int32), ("record_tree_threshold", ctypes.c_int32),
        ("record_tree_target_weight", ctypes.c_float),
    ]


class SelfplayConfig(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_int32), ("y", ctypes.c_int32), ("win_len", ctypes.c_int32),
        ("num_games", ctypes.c_int32), ("node_cap", ctypes.c_int32), ("row_capacity", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("slot_base", ctypes.c_int32), ("use_fake_net", ctypes.c_int32),
        ("commit_interval", ctypes.c_int32),
        ("model_path", ctypes.c_char_p),
        ("search", SearchParams),
        ("nn_cache_log2", ctypes.c_int32),
        ("nn_batch_cap", ctypes.c_int32),
        ("nn_precision", ctypes.c_int32),
        ("start_stagger", ctypes.c_int32),
        ("engines_per_device", ctypes.c_int32),
    ]


class SelfplayStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ["rounds", "playouts", "nn_evals", "moves", "games_finished", "rows_written", "rows_pending",
                 "rows_dropped", "games_dropped", "errors", "tree_levels", "tree_children", "errors_node_pool",
                 "errors_edge_pool", "edge_pool_peak", "edge_pool_cap", "nn_precision", "nn_audits",
                 "nn_audit_switches"]] + [("nn_audit_max_diff", ctypes.c_double)]


# Every symbol include/katacoffee.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "coffee_last_error", "coffee_abi_version", "coffee_device_count", "coffee_set_device", "coffee_device_compute_units", "coffee_malloc",
    "coffee_free", "coffee_memcpy", "coffee_synchronize", "coffee_rules_batch", "coffee_play_batch",
    "coffee_encode_batch", "coffee_model_write_random", "coffee_model_flops", "coffee_nn_create",
    "coffee_nn_forward", "coffee_nn_forward2", "coffee_nn_destroy", "coffee_nn_create2", "coffee_nn_is_fused", "coffee_nn_precision", "coffee_fake_net", "coffee_search_params_default",
    "coffee_selfplay_create", "coffee_selfplay_step", "coffee_selfplay_sync", "coffee_selfplay_stats_get",
    "coffee_selfplay_drain_rows", "coffee_selfplay_drain_games", "coffee_selfplay_set_model",
    "coffee_selfplay_stage_rows", "coffee_selfplay_row_capacity", "coffee_row_bytes", "coffee_selfplay_stream",
    "coffee_selfplay_set_model_bytes",
    "coffee_selfplay_destroy", "coffee_selfplay_game_info",
    "coffee_selfplay_game_tree", "coffee_selfplay_root_policy", "coffee_debug_cdf_table", "coffee_debug_zobrist",
    "coffee_selfplay_enable_timing", "coffee_selfplay_kernel_time", "coffee_selfplay_timed_nn_evals",
    "coffee_write_npz",
]


def build(jobs=8):
    """Compile libkatacoffee.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-j%d" % jobs, "-C", CSRC], check=True)


def lib():
    """The loaded C-ABI library.  Raises if it was not built — there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CoffeeError("libkatacoffee.so not built (run katacoffee_amd.build()); no CPU fallback exists")
        # One HIP runtime per process: torch's libraries ask for "libamdhip64.so" while
        # ours asks for the SONAME "libamdhip64.so.7".  Loading torch first lets our
        # request resolve to torch's already-loaded copy; the reverse order would load
        # two runtimes, and ours would then see no device.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        # KATACOFFEE_LIB: an alternative build of the same library (profiling builds)
        L = ctypes.CDLL(os.environ.get("KATACOFFEE_LIB", LIB_PATH))
        L.coffee_last_error.restype = ctypes.c_char_p
        L.coffee_model_write_random.argtypes = [ctypes.c_char_p, c_u64, ctypes.c_char_p]
        L.coffee_model_flops.argtypes = [ctypes.c_char_p, c_i, c_p]
        L.coffee_nn_create.argtypes = [ctypes.c_char_p, c_i, c_i, c_i, c_p]
        L.coffee_nn_create2.argtypes = [ctypes.c_char_p, c_i, c_i, c_i, c_i, c_p]
        L.coffee_nn_is_fused.argtypes = [c_p, c_p]
        if hasattr(L, "coffee_nn_precision"):  # (absent in round-4 builds run as A/B references)
            L.coffee_nn_precision.argtypes = [c_p, c_p, c_p]
        L.coffee_nn_forward.argtypes = [c_p, c_i, c_p, c_p, c_p]
        L.coffee_nn_forward2.argtypes = [c_p, c_i, c_p, c_p, c_p, c_p]
        L.coffee_nn_destroy.argtypes = [c_p]
        L.coffee_fake_net.argtypes = [c_i, c_i, c_i, c_i, c_p, c_p, c_p]
        L.coffee_rules_batch.argtypes = [c_i, c_i, c_i, c_i] + [c_p] * 7
        L.coffee_play_batch.argtypes = [c_i, c_i, c_i, c_i] + [c_p] * 12
        L.coffee_encode_batch.argtypes = [c_i, c_i, c_i, c_i] + [c_p] * 8
        L.coffee_search_params_default.argtypes = [c_p]
        L.coffee_search_params_default.restype = None
        L.coffee_selfplay_create.argtypes = [c_p, c_p]
        L.coffee_selfplay_step.argtypes = [c_p, c_i, c_p]
        L.coffee_selfplay_sync.argtypes = [c_p]
        L.coffee_selfplay_stats_get.argtypes = [c_p, c_p]
        L.coffee_selfplay_drain_rows.argtypes = [c_p, c_i] + [c_p] * 7
        L.coffee_selfplay_drain_games.argtypes = [c_p, c_i, c_p, c_p, c_p]
        L.coffee_selfplay_stage_rows.argtypes = [c_p, c_p, c_i, c_p, c_i]
        L.coffee_selfplay_row_capacity.argtypes = [c_p, c_p]
        L.coffee_row_bytes.argtypes = [c_i, c_i, c_p]
        L.coffee_selfplay_stream.argtypes = [c_p, c_p]
        L.coffee_selfplay_set_model.argtypes = [c_p, ctypes.c_char_p]
        L.coffee_selfplay_set_model_bytes.argtypes = [c_p, c_p, c_u64]
        L.coffee_selfplay_destroy.argtypes = [c_p]
        L.coffee_selfplay_game_info.argtypes = [c_p, c_i, c_p]
        L.coffee_selfplay_game_tree.argtypes = [c_p, c_i, c_i, c_p, c_p, c_p]
        L.coffee_selfplay_root_policy.argtypes = [c_p, c_i, c_p]
        L.coffee_selfplay_enable_timing.argtypes = [c_p, c_i]
        L.coffee_selfplay_kernel_time.argtypes = [c_p, c_i, c_p, c_p]
        L.coffee_selfplay_timed_nn_evals.argtypes = [c_p, c_p]
        L.coffee_debug_cdf_table.argtypes = [c_i, c_i, c_i, c_p]
        L.coffee_debug_zobrist.argtypes = [c_i, c_i, c_i] + [c_p] * 5
        L.coffee_write_npz.argtypes = [ctypes.c_char_p, c_i, c_i, c_i] + [c_p] * 5
        _lib = L
    return _lib


def check(rc):
    if rc != COFFEE_OK:
        msg = lib().coffee_last_error()
        raise CoffeeError("libkatacoffee error %d: %s" % (rc, msg.decode() if msg else ""))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def default_search_params(**over):
    p = SearchParams()
    lib().coffee_search_params_default(ctypes.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


# ---------------------------------------------------------------------------
# Batched rules / encoder / network through device tensors.

def _torch_cuda():
    import torch
    if not torch.cuda.is_available():
        raise CoffeeError("no GPU visible: the HIP path is the only implementation")
    return torch


def _dev(torch, a, dtype=None):
    a = np.ascontiguousarray(a if dtype is None else np.asarray(a, dtype=dtype))
    return torch.from_numpy(a).to("cuda")


def _dp(t):
    return ctypes.c_void_p(t.data_ptr())


def _sync(torch):
    torch.cuda.synchronize()


def rules_batch(X, Y, W, cells, last_cell, last_dir, pla):
    """Legal-move masks [n][4A] u8 and has-legal flags [n] u8 (Board::isLegal board.cpp:185-227)."""
    torch = _torch_cuda()
    n = len(pla)
    A = X * Y
    dc, dl, dd, dp_ = (_dev(torch, cells, np.uint8), _dev(torch, last_cell, np.int8), _dev(torch, last_dir, np.int8),
                       _dev(torch, pla, np.uint8))
    legal = torch.zeros((n, 4 * A), dtype=torch.uint8, device="cuda")
    has = torch.zeros(n, dtype=torch.uint8, device="cuda")
    _sync(torch)
    check(lib().coffee_rules_batch(X, Y, W, n, _dp(dc), _dp(dl), _dp(dd), _dp(dp_), _dp(legal), _dp(has), None))
    _sync(torch)
    return legal.cpu().numpy(), has.cpu().numpy()


def play_batch(X, Y, W, cells, last_cell, last_dir, pla, move):
    torch = _torch_cuda()
    n = len(pla)
    A = X * Y
    ins = [_dev(torch, cells, np.uint8), _dev(torch, last_cell, np.int8), _dev(torch, last_dir, np.int8),
           _dev(torch, pla, np.uint8), _dev(torch, move, np.int32)]
    out_cells = torch.zeros((n, A), dtype=torch.uint8, device="cuda")
    fin = torch.zeros(n, dtype=torch.uint8, device="cuda")
    win = torch.zeros(n, dtype=torch.uint8, device="cuda")
    mr = torch.zeros(n, dtype=torch.int32, device="cuda")
    ph = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    sh = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    _sync(torch)
    check(lib().coffee_play_batch(X, Y, W, n, *[_dp(t) for t in ins], _dp(out_cells), _dp(fin), _dp(win), _dp(mr),
                                  _dp(ph), _dp(sh), None))
    _sync(torch)
    u = lambda t: t.cpu().numpy().view(np.uint64)
    return (out_cells.cpu().numpy(), fin.cpu().numpy(), win.cpu().numpy(), mr.cpu().numpy(), u(ph), u(sh))


def encode_batch(X, Y, W, cells, hist_cell, hist_dir, pla, sym, want_planes=True):
    """Packed V1 rows [n][ceil(15A/64)] u64 and optionally planes [n][15][A] f32."""
    torch = _torch_cuda()
    n = len(pla)
    A = X * Y
    words = (NUM_SPATIAL * A + 63) // 64
    ins = [_dev(torch, cells, np.uint8), _dev(torch, hist_cell, np.int8), _dev(torch, hist_dir, np.int8),
           _dev(torch, pla, np.uint8), _dev(torch, sym, np.int32)]
    packed = torch.zeros((n, words), dtype=torch.int64, device="cuda")
    planes = torch.zeros((n, NUM_SPATIAL, A), dtype=torch.float32, device="cuda") if want_planes else None
    _sync(torch)
    check(lib().coffee_encode_batch(X, Y, W, n, *[_dp(t) for t in ins], _dp(packed),
                                    _dp(planes) if planes is not None else None, None))
    _sync(torch)
    pk = packed.cpu().numpy().view(np.uint64)
    return pk, (planes.cpu().numpy() if planes is not None else None)


def write_random_model(arch, seed, path):
    check(lib().coffee_model_write_random(arch.encode(), seed, path.encode()))


def model_flops(path, area):
    f = ctypes.c_double()
    check(lib().coffee_model_flops(path.encode(), area, ctypes.byref(f)))
    return f.value


class Network:
    """NeuralNet compute handle (nninterface.h createComputeHandle / getOutput).

    precision (include/katacoffee.h COFFEE_NN_*): "default" (the 1e-3-of-fp32 path:
    "corrected" where the fused kernel covers the net, "accurate" otherwise), "corrected"
    (fp16 products + block-scaled e4m3 cross terms), "accurate" (fp16 hi/lo operand pairs:
    within 1e-3 of fp32 for any net), "fast" (fp16 operands; the fused kernel where it
    covers the net) or "fast-layered" (fp16 operands on the per-convolution kernels)."""

    def __init__(self, model_path, X, Y, W, precision="default"):
        self.X, self.Y, self.W = X, Y, W
        self.h = ctypes.c_void_p()
        check(lib().coffee_nn_create2(model_path.encode(), X, Y, W, PRECISIONS[precision], ctypes.byref(self.h)))

    @property
    def fused(self):
        f = ctypes.c_int()
        check(lib().coffee_nn_is_fused(self.h, ctypes.byref(f)))
        return bool(f.value)

    @property
    def precision(self):
        """(name of the precision the handle runs, calibration difference of the default
        precision's corrected-vs-accurate check or 0.0) -- coffee_nn_precision."""
        p, e = ctypes.c_int(), ctypes.c_float()
        check(lib().coffee_nn_precision(self.h, ctypes.byref(p), ctypes.byref(e)))
        return PRECISION_NAMES[p.value], float(e.value)

    def forward_device(self, n, packed_dev, out_dev, stream=None):
        check(lib().coffee_nn_forward(self.h, n, _dp(packed_dev), _dp(out_dev), stream))

    def forward(self, packed):
        """packed [n][words] u64 (host) -> [n][P+4] f32 (host)."""
        torch = _torch_cuda()
        n = packed.shape[0]
        P = 4 * self.X * self.Y
        din = _dev(torch, np.ascontiguousarray(packed).view(np.int64))
        out = torch.zeros((n, P + 4), dtype=torch.float32, device="cuda")
        _sync(torch)
        self.forward_device(n, din, out)
        _sync(torch)
        return out.cpu().numpy()

    def forward_canonical(self, packed, sym):
        """NeuralNet::getOutput (eigenbackend.cpp:1776-1796): packed [n][words] u64 rows
        encoded with symmetries sym [n] -> [n][P+4] f32 with the policy logits in the
        canonical frame (coffee_nn_forward2)."""
        torch = _torch_cuda()
        n = packed.shape[0]
        P = 4 * self.X * self.Y
        din = _dev(torch, np.ascontiguousarray(packed).view(np.int64))
        dsym = _dev(torch, sym, np.int32)
        out = torch.zeros((n, P + 4), dtype=torch.float32, device="cuda")
        _sync(torch)
        check(lib().coffee_nn_forward2(self.h, n, _dp(din), _dp(dsym), _dp(out), None))
        _sync(torch)
        return out.cpu().numpy()

    def close(self):
        if self.h:
            lib().coffee_nn_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fake_net(X, Y, W, packed):
    torch = _torch_cuda()
    n = packed.shape[0]
    P = 4 * X * Y
    din = _dev(torch, np.ascontiguousarray(packed).view(np.int64))
    out = torch.zeros((n, P + 4), dtype=torch.float32, device="cuda")
    _sync(torch)
    check(lib().coffee_fake_net(X, Y, W, n, _dp(din), _dp(out), None))
    _sync(torch)
    return out.cpu().numpy()


def cdf_table(X=5, Y=5, W=4):
    out = np.zeros(2000, np.float32)
    check(lib().coffee_debug_cdf_table(X, Y, W, _ptr(out)))
    return out


def row_bytes(X, Y):
    """Bytes of one packed row (coffee_row_bytes; katacoffee_amd.rows.row_bytes)."""
    b = ctypes.c_int()
    check(lib().coffee_row_bytes(X, Y, ctypes.byref(b)))
    return b.value


def write_npz(path, rows, X, Y):
    """Training rows -> .npz in the reference's format (native writer)."""
    n = len(rows["globalInputNC"])
    arrs = [np.ascontiguousarray(rows[k], dtype=t) for k, t in
            [("binaryInputNCHWPacked", np.uint8), ("globalInputNC", np.float32), ("policyTargetsNCMove", np.int16),
             ("globalTargetsNC", np.float32), ("valueTargetsNCHW", np.int8)]]
    check(lib().coffee_write_npz(path.encode(), n, X, Y, *[_ptr(a) for a in arrs]))


def zobrist_tables(X, Y, W):
    A = X * Y
    out = dict(board=np.zeros((A, 3, 2), np.uint64), board2=np.zeros((A, 4, 2), np.uint64),
               player=np.zeros((3, 2), np.uint64), init=np.zeros(2, np.uint64), game_over=np.zeros(2, np.uint64))
    check(lib().coffee_debug_zobrist(X, Y, W, *[_ptr(out[k]) for k in ["board", "board2", "player", "init",
                                                                          "game_over"]]))
    return out


class Selfplay:
    """One device's self-play engine (games [slot_base, slot_base + num_games))."""

    def __init__(self, X=5, Y=5, W=4, num_games=4096, max_visits=600, seed=1, slot_base=0, model_path=None,
                 node_cap=0, row_capacity=0, commit_interval=0, nn_cache_log2=0, nn_batch_cap=0, nn_precision="default",
                 start_stagger=0, engines_per_device=0, **search_over):
        _torch_cuda()
        self.X, self.Y, self.W = X, Y, W
        self.A, self.P = X * Y, 4 * X * Y
        self.num_games = num_games
        cfg = SelfplayConfig()
        cfg.x, cfg.y, cfg.win_len = X, Y, W
        cfg.num_games = num_games
        cfg.node_cap = node_cap
        cfg.row_capacity = row_capacity
        cfg.seed = seed
        cfg.slot_base = slot_base
        cfg.use_fake_net = 1 if model_path is None else 0
        cfg.commit_interval = commit_interval
        cfg.nn_cache_log2 = nn_cache_log2
        cfg.nn_batch_cap = nn_batch_cap
        cfg.nn_precision = PRECISIONS[nn_precision]
        cfg.start_stagger = start_stagger
        cfg.engines_per_device = engines_per_device
        self._model = model_path.encode() if model_path else None
        cfg.model_path = self._model
        cfg.search = default_search_params(max_visits=max_visits, **search_over)
        self.cfg = cfg
        self.h = ctypes.c_void_p()
        check(lib().coffee_selfplay_create(ctypes.byref(cfg), ctypes.byref(self.h)))

    def step(self, rounds, stream=None):
        check(lib().coffee_selfplay_step(self.h, rounds, stream))

    def sync(self):
        check(lib().coffee_selfplay_sync(self.h))

    def stats(self):
        s = SelfplayStats()
        check(lib().coffee_selfplay_stats_get(self.h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in SelfplayStats._fields_}

    def drain_rows(self, max_rows=1 << 30):
        st = self.stats()
        n = min(max_rows, st["rows_pending"])
        A, P, pb = self.A, self.P, (self.A + 7) // 8
        rows = {
            "binaryInputNCHWPacked": np.zeros((n, NUM_SPATIAL, pb), np.uint8),
            "globalInputNC": np.zeros((n, 1), np.float32),
            "policyTargetsNCMove": np.zeros((n, 2, P), np.int16),
            "globalTargetsNC": np.zeros((n, 64), np.float32),
            "valueTargetsNCHW": np.zeros((n, 5, self.Y, self.X), np.int8),
            "meta": np.zeros((n, 4), np.int32),
        }
        got = ctypes.c_int()
        order = ["binaryInputNCHWPacked", "globalInputNC", "policyTargetsNCMove", "globalTargetsNC",
                 "valueTargetsNCHW", "meta"]
        check(lib().coffee_selfplay_drain_rows(self.h, n, *[_ptr(rows[k]) for k in order], ctypes.byref(got)))
        assert got.value == n
        return rows

    def row_capacity(self):
        n = ctypes.c_int()
        check(lib().coffee_selfplay_row_capacity(self.h, ctypes.byref(n)))
        return n.value

    def stream_ptr(self):
        """The engine's hipStream_t (for torch.cuda.ExternalStream)."""
        p = ctypes.c_void_p()
        check(lib().coffee_selfplay_stream(self.h, ctypes.byref(p)))
        return p.value

    def stage_rows(self, dst, count, discard_games=True):
        """Device-resident row hand-off (coffee_selfplay_stage_rows), enqueued on the
        engine's stream: dst a device uint8 tensor [>= row_capacity][row_bytes], count a
        pinned host int64 tensor element (filled asynchronously)."""
        assert dst.is_cuda and dst.dtype.itemsize == 1 and dst.is_contiguous()
        # the kernel writes up to dst.shape[0] whole rows: a buffer of another shape or on
        # another device would be written out of bounds
        assert dst.dim() == 2 and dst.shape[1] == row_bytes(self.X, self.Y), \
            "dst must be [rows][row_bytes(X, Y)] uint8, got %s" % (tuple(dst.shape),)
        import torch
        assert dst.device.index == torch.cuda.current_device(), "dst must be on the engine's (current) device"
        assert count.is_pinned() and count.dtype.itemsize == 8
        check(lib().coffee_selfplay_stage_rows(self.h, ctypes.c_void_p(dst.data_ptr()), dst.shape[0],
                                               ctypes.c_void_p(count.data_ptr()), 1 if discard_games else 0))

    def drain_games(self, max_games=1 << 20):
        """Finished-game records: header [g][4] i32 (slot, game number, moves, winner)
        and moves [g][A][2] u8 (cell, direction; 0xFF past the last move)."""
        cap = min(max_games, 2 * self.num_games)
        header = np.zeros((cap, 4), np.int32)
        moves = np.zeros((cap, self.A, 2), np.uint8)
        got = ctypes.c_int()
        check(lib().coffee_selfplay_drain_games(self.h, cap, _ptr(header), _ptr(moves), ctypes.byref(got)))
        return header[:got.value], moves[:got.value]

    def set_model(self, model_path):
        """Hot reload: every later round of every game uses this network."""
        self._model = model_path.encode()
        check(lib().coffee_selfplay_set_model(self.h, self._model))

    def set_model_bytes(self, data):
        """Hot reload from a CFNN image in memory (bytes / uint8 array), e.g. weights
        broadcast from rank 0 (katacoffee_amd.weights.broadcast_model)."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        check(lib().coffee_selfplay_set_model_bytes(self.h, _ptr(buf), buf.size))

    def game_info(self, slot):
        info = np.zeros(16, np.int64)
        check(lib().coffee_selfplay_game_info(self.h, slot, _ptr(info)))
        keys = ["phase", "rootK", "liveCount", "rootIdx", "gameNum", "turn", "pla", "finished", "winner",
                "playouts", "nnEvals", "moves", "gamesFinished", "lastCell", "lastDir", "rngCtr"]
        return dict(zip(keys, info.tolist()))

    def game_tree(self, slot, max_nodes=4096):
        nodes = np.zeros((max_nodes, 24), np.uint32)
        edges = np.zeros((max_nodes, self.P, 3), np.uint32)
        n = ctypes.c_int()
        check(lib().coffee_selfplay_game_tree(self.h, slot, max_nodes, _ptr(nodes), _ptr(edges), ctypes.byref(n)))
        return nodes[:n.value], edges[:n.value]

    def root_policy(self, slot):
        out = np.zeros(self.P, np.float32)
        check(lib().coffee_selfplay_root_policy(self.h, slot, _ptr(out)))
        return out

    def enable_timing(self, every=1):
        """Time every `every`-th launch of each kernel group with HIP events (0 = off)."""
        check(lib().coffee_selfplay_enable_timing(self.h, int(every)))

    def timed_nn_evals(self):
        """Network evaluations performed by the timed network launches."""
        n = ctypes.c_uint64()
        check(lib().coffee_selfplay_timed_nn_evals(self.h, ctypes.byref(n)))
        return n.value

    def kernel_time(self, which):
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        check(lib().coffee_selfplay_kernel_time(self.h, which, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def close(self):
        if self.h:
            lib().coffee_selfplay_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
