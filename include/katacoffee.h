/* katacoffee.h — C ABI of the MI355X Coffee self-play engine (libkatacoffee.so).
 *
 * This is the drop-in boundary of SURVEY.md §8(b): the in-process surface that
 * replaces the reference's rules / encoder / NN-backend / self-play hot path.
 * Every entry point:
 *   - is extern "C", takes plain pointers and sizes, never throws;
 *   - returns 0 on success and a negative COFFEE_E* code on failure, with the
 *     message in coffee_last_error() (thread-local) — the reference reports the
 *     same failures as C++ StringError exceptions (eigenbackend.cpp:1602-1605);
 *   - takes DEVICE pointers for bulk data unless the parameter says "host",
 *     and an optional hipStream_t (`stream`, NULL = the default stream).
 * Handles are single-thread objects, like NeuralNet::ComputeHandle
 * (nninterface.h:18-20) and Search (search.h:159-165); use one handle per GPU.
 *
 * Board geometry: X columns x Y rows, 2 <= X, Y <= 10; cell = y*X + x; A = X*Y.
 * Move encoding ("pos"): pos = dir*A + cell, dir 0=N 1=W 2=NW 3=NE (board.h:41-47);
 * P = 4A.  Colours: 0 empty, 1 black, 2 white.  Player 1 moves first.
 * lastDir 4 = NONE (no previous move), lastCell -1 = none.
 */
#ifndef KATACOFFEE_H
#define KATACOFFEE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COFFEE_OK 0
#define COFFEE_EINVAL (-1)   /* bad argument / unsupported geometry or model */
#define COFFEE_EHIP (-2)     /* HIP runtime error */
#define COFFEE_EIO (-3)      /* file I/O or format error */
#define COFFEE_EINTERNAL (-4)

#define COFFEE_NUM_SPATIAL 15 /* V1 planes (README "V1", SPEC a6) */
#define COFFEE_NUM_GLOBAL_TARGETS 64

/* Last error message of the calling thread ("" if none). */
const char* coffee_last_error(void);
/* ABI version (major*100 + minor). */
int coffee_abi_version(void);

/* ---- device memory helpers (so callers need no HIP headers) ---- */
int coffee_device_count(int* count);
int coffee_set_device(int device);
/* Compute units of `device` (the fused network runs one workgroup per CU: a host that
   runs several self-play engines on one device splits cus x 8 rows of batch cap
   between them, as the CLI does for numNNServerThreadsPerModel). */
int coffee_device_compute_units(int device, int* cus);
int coffee_malloc(void** dev_ptr, uint64_t bytes);
int coffee_free(void* dev_ptr);
/* kind: 0 host->device, 1 device->host, 2 device->device */
int coffee_memcpy(void* dst, const void* src, uint64_t bytes, int kind);
int coffee_synchronize(void);

/* ---- rules (replaces Board::isLegal board.cpp:185-227,
 *      Board::playMoveAssumeLegal board.cpp:427-435 + BoardHistory::makeBoardMoveAssumeLegal
 *      boardhistory.cpp:157-176, Board::maxConsecutives board.cpp:315-335,
 *      Board pos_hash board.cpp:134-178, GraphHash::getStateHash graphhash.cpp:3-34) ---- */

/* n positions.  cells [n][A] u8 colours; last_cell/last_dir [n] int8; pla [n] u8.
 * legal  [n][P] u8 (1 = legal move for pla)        (out)
 * has_legal [n] u8 (0 = no legal move: SPEC B16 draw) (out) */
int coffee_rules_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* last_cell,
                       const int8_t* last_dir, const uint8_t* pla, uint8_t* legal, uint8_t* has_legal, void* stream);

/* Plays move[i] (pos, assumed legal) for pla[i].  Outputs:
 * out_cells [n][A]; finished/winner [n] u8 (winner 0 = none/draw); max_run [n] i32
 * (longest run through the move); pos_hash [n][2] u64 (Board::pos_hash after);
 * state_hash [n][2] u64 (transposition key: pos_hash ^ next player ^ last move ^ game over). */
int coffee_play_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* last_cell,
                      const int8_t* last_dir, const uint8_t* pla, const int32_t* move, uint8_t* out_cells,
                      uint8_t* finished, uint8_t* winner, int32_t* max_run, uint64_t* pos_hash,
                      uint64_t* state_hash, void* stream);

/* ---- V1 encoder (replaces NNInputs::fillRowV1 nninputs.cpp:508-657 with SPEC a6,
 *      symmetry SymmetryHelpers nninputs.cpp:252-433) ---- */

/* hist_cell/hist_dir [n][5]: the last five moves, [0] most recent (-1 / 4 = none).
 * sym [n] in 0..7 (bit0 flip y, bit1 flip x, bit2 transpose; transpose ignored when X != Y).
 * packed [n][ceil(15A/64)] u64: bit i = plane*A + symcell      (out, required)
 * planes [n][15][A] f32 (NCHW, symmetric frame)                  (out, optional: NULL)
 * The global input is the single value win_len. */
int coffee_encode_batch(int x, int y, int win_len, int n, const uint8_t* cells, const int8_t* hist_cell,
                        const int8_t* hist_dir, const uint8_t* pla, const int32_t* sym, uint64_t* packed,
                        float* planes, void* stream);

/* ---- network (replaces the NeuralNet:: backend interface nninterface.h:31-171:
 *      loadModelFile / createComputeHandle / getOutput / free*) ---- */

typedef struct coffee_nn coffee_nn;

/* Writes a seeded random-init CFNN model file ("b6c96", "b10c128", "b18c384nbt",
 * "b2c32", "b2c32nbt"; modelconfigs.py:129/156/887). */
int coffee_model_write_random(const char* arch, uint64_t seed, const char* path /* host */);
/* FLOPs per evaluation (2 x MACs) of a CFNN model at area A. */
int coffee_model_flops(const char* path, int area, double* flops);

/* Loads a CFNN model and prepares device weights for boards X x Y with win length W
 * (NeuralNet::loadModelFile + createComputeHandle, nninterface.h:42-109).
 * coffee_nn_create = coffee_nn_create2(..., COFFEE_NN_DEFAULT, ...). */
int coffee_nn_create(const char* model_path, int x, int y, int win_len, coffee_nn** out);
/* precision (the reference's useFP16 switch, nninterface.h:76-88; its default, Auto,
 * setup.cpp:240-248, maps here to the path that meets the north-star 1e-3 of fp32):
 *   COFFEE_NN_DEFAULT       (0) the 1e-3 path: where the fused kernel covers the net (b6c96
 *                           @ 5x5), CORRECTED if a load-time calibration batch (corrected vs
 *                           accurate on 256 seeded positions) differs by at most 2.5e-4 and
 *                           flags no board, else ACCURATE; the layered split (ACCURATE)
 *                           kernels for every other net (coffee_nn_precision reports it)
 *   COFFEE_NN_ACCURATE      fp16 hi/lo operand pairs on three MFMAs (the fused kernel's
 *                           split instance where it covers the net, the layered kernels
 *                           otherwise): logits within ~1e-5 of the fp32 (Eigen-semantics) forward
 *   COFFEE_NN_FAST_LAYERED  fp16 operands on the layered kernels (any architecture)
 *   COFFEE_NN_CORRECTED     fp16 products plus the two fp16-rounding cross terms on
 *                           block-scaled e4m3 MFMAs (twice the fp16 MFMA work): the weights'
 *                           e4m3 operands carry one power-of-two exponent per convolution
 *                           (its largest |w| lands in (224, 448], so no weight saturates);
 *                           activations are unscaled, and a board with a convolution input
 *                           past e4m3's 448 is flagged and re-evaluated on the ACCURATE
 *                           instance in a second launch.  A product is good to ~2^-14, so
 *                           the error grows with the logits: 7e-4 of fp32 on a net trained
 *                           200 steps (logits ~20), ~1e-3 after 1000 -- not
 *                           a 1e-3 path for every net, hence DEFAULT's calibration.  The
 *                           fused kernel where it covers the net, else as ACCURATE
 *   COFFEE_NN_ACCURATE_NB2  ACCURATE on the 2-board bordered fused instance (A/B reference
 *                           of the borderless 5-board one; same results bit for bit)
 *   COFFEE_NN_FAST          fp16 MFMA operands, f32 accumulation and residual trunk (the
 *                           fused single-launch kernel where it covers the net, the layered
 *                           kernels otherwise): ~1e-3 of the largest logit off fp32, which
 *                           misses the 1e-3 absolute bound on trained nets */
#define COFFEE_NN_DEFAULT 0
#define COFFEE_NN_ACCURATE 1
#define COFFEE_NN_FAST_LAYERED 2
#define COFFEE_NN_CORRECTED 3
#define COFFEE_NN_ACCURATE_NB2 4
#define COFFEE_NN_FAST 5
int coffee_nn_create2(const char* model_path, int x, int y, int win_len, int precision, coffee_nn** out);
/* 1 when the handle runs the fused single-launch kernel, 0 for the layered kernels. */
int coffee_nn_is_fused(coffee_nn* h, int* fused);
/* The precision the handle runs (COFFEE_NN_*, COFFEE_NN_DEFAULT resolved: CORRECTED, or
 * ACCURATE when the corrected instance's logits on a fixed calibration batch -- 256
 * positions of seeded random legal play -- differ from the accurate instance's by more than
 * 2.5e-4, a quarter of the north-star bound; ACCURATE / FAST_LAYERED on the layered kernels)
 * and that calibration difference (*calib_err, 0 when no check ran; may be NULL). */
int coffee_nn_precision(coffee_nn* h, int* precision, float* calib_err);
/* in: packed V1 rows [n][ceil(15A/64)] (coffee_encode_batch layout);
 * out: [n][P+4] f32 = policy logits [4][A] (symmetric frame, dir-major), value logits
 * (win, loss) from the side to move, misc[2].  fp16 MFMA operands (see precision),
 * f32 accumulation. */
int coffee_nn_forward(coffee_nn* h, int n, const uint64_t* in, float* out, void* stream);
/* NeuralNet::getOutput's contract (eigenbackend.cpp:1776-1796): as coffee_nn_forward, with
 * sym [n] i32 (device) = the symmetry each row was encoded with (coffee_encode_batch's
 * sym); the policy logits come back in the CANONICAL frame, the inverse symmetry applied
 * per SPEC B12 (cells un-flipped / un-transposed and the directions mapped back: a one-axis
 * flip swaps NW<->NE, a transpose swaps N<->W), as copyOutputsWithSymmetry does.  Value
 * logits (win, loss; side to move) and misc[2] are symmetry-free and unchanged.  The
 * NNEvaluator-side post-processing (legal mask, softmax, white perspective;
 * nneval.cpp:702-844) stays with the caller, as in the reference. */
int coffee_nn_forward2(coffee_nn* h, int n, const uint64_t* in, const int32_t* sym, float* out, void* stream);
int coffee_nn_destroy(coffee_nn* h);

/* The deterministic stand-in network (oracle fakeNet), same I/O as coffee_nn_forward. */
int coffee_fake_net(int x, int y, int win_len, int n, const uint64_t* in, float* out, void* stream);

/* ---- self-play engine (replaces Play::runGame play.cpp:1146-1701 driving
 *      Search::runWholeSearch search.cpp:361-509 and TrainingWriteBuffers
 *      trainingwrite.cpp:316-565 for numGameThreads games) ---- */

/* SearchParams (searchparams.h) restricted to Coffee self-play; defaults =
 * cpp/configs/training/selfplay1.cfg with benchmark settings. */
typedef struct coffee_search_params {
  int32_t max_visits;
  float cpuct_exploration, cpuct_exploration_log, cpuct_exploration_base;
  float fpu_reduction_max, root_fpu_reduction_max, fpu_loss_prop, root_fpu_loss_prop;
  int32_t fpu_parent_weight_by_visited_policy;
  float fpu_parent_weight_by_visited_policy_pow;
  float value_weight_exponent;
  int32_t root_noise_enabled;
  float root_dirichlet_noise_total_concentration, root_dirichlet_noise_weight;
  float root_policy_temperature, root_policy_temperature_early;
  float root_desired_per_child_visits_coeff;
  int32_t root_num_symmetries_to_sample;
  float chosen_move_temperature, chosen_move_temperature_early, chosen_move_temperature_halflife;
  float chosen_move_subtract, chosen_move_prune;
  int32_t use_lcb_for_selection;
  float lcb_stdevs, min_visit_prop_for_lcb;
  float subtree_value_bias_factor, subtree_value_bias_weight_exponent, subtree_value_bias_free_prop;
  int32_t use_graph_search;
  /* PlaySettings (playsettings.cpp): per-move search limits (getSearchLimitsThisMove
   * play.cpp:871-1004) and row weighting (play.cpp:1470-1697).  Defaults are the
   * benchmark mode of SURVEY 8d (all off); selfplay1.cfg values in comments. */
  float cheap_search_prob;           /* 0.75 */
  int32_t cheap_search_visits;       /* 100 */
  float cheap_search_target_weight;  /* 0.0 */
  int32_t reduce_visits;             /* 1 */
  float reduce_visits_threshold;     /* 0.9 */
  int32_t reduce_visits_threshold_lookback; /* 3 */
  int32_t reduced_visits_min;        /* 100 */
  float reduced_visits_weight;       /* 0.1 */
  float policy_surprise_data_weight; /* 0.5 */
  float value_surprise_data_weight;  /* 0.1 */
  /* opening moves sampled from the raw policy before the searched game
   * (initializeGameUsingPolicy playutils.cpp:147-176) */
  int32_t init_games_with_policy;    /* 1 */
  float policy_init_area_prop;       /* 0.04: mean number of moves / board area */
  float policy_init_area_temperature;/* 1.0 */
  /* forks (Play::maybeForkGame play.cpp:1741-1840): after a game, with these
   * probabilities the slot's next game starts from a replayed position of it plus the
   * best (by the value head) of a few random legal moves */
  float early_fork_game_prob;            /* 0.04 */
  float early_fork_game_expected_move_prop; /* 0.025 */
  float fork_game_prob;                  /* 0.01 */
  int32_t fork_game_min_choices;         /* 3 */
  int32_t early_fork_game_max_choices;   /* 12 */
  int32_t fork_game_max_choices;         /* 36 */
  /* side positions (play.cpp:1328-1345, :1576-1662): after a searched move, with this
   * probability a refutation position (the root policy's alternative to the played
   * move) is queued and searched after the game; one row each */
  float side_position_prob;              /* 0.02 */
  /* tree positions (recordTreePositions play.cpp:710-860, :1347-1361, :1612-1628): after
   * a searched move (or side position), positions of its search tree up to 5 moves deep
   * reached only through the mover's most-visited moves, from nodes with at least
   * record_tree_threshold visits, are written as side rows with weight
   * record_tree_target_weight (<= 1).  PlaySettings fields with these defaults
   * (playsettings.cpp:14); the reference's selfplay config loader does not read them */
  int32_t record_tree_positions;         /* 0 */
  int32_t record_tree_threshold;         /* 0 */
  float record_tree_target_weight;       /* 0.0 */
} coffee_search_params;

void coffee_search_params_default(coffee_search_params* p);

typedef struct coffee_selfplay_config {
  int32_t x, y, win_len;
  int32_t num_games;     /* concurrent games on this device (numGameThreads) */
  int32_t node_cap;      /* per-game node pool; 0 = max(2048, 3*max_visits) */
  int32_t row_capacity;  /* device row buffer capacity; 0 = 4*num_games*A */
  uint64_t seed;         /* run seed (gameSeedBase) */
  int32_t slot_base;     /* global index of slot 0 (rank * num_games) */
  int32_t use_fake_net;  /* 1 = coffee_fake_net instead of the model */
  int32_t commit_interval; /* rounds between move-commit launches (0 = 8); 1 commits in
                              the round the root reaches max_visits, like the oracle */
  const char* model_path;/* CFNN model (host string), ignored with use_fake_net */
  coffee_search_params search;
  int32_t nn_cache_log2; /* NN evaluation cache entries = 2^nn_cache_log2 (selfplay1.cfg
                            nnCacheSizePowerOfTwo = 21); 0 disables (SPEC a7) */
  int32_t nn_batch_cap;  /* rows per network launch; leaves past it wait for the next round,
                            ahead of new ones.  0 = one full wave of network workgroups
                            (compute units x 8 boards: 2048 on MI355X, / engines_per_device)
                            for the fused kernel, unbounded for the layered kernels */
  int32_t nn_precision;  /* COFFEE_NN_DEFAULT (0: the 1e-3 path) / _CORRECTED / _ACCURATE /
                            _FAST / _FAST_LAYERED */
  int32_t start_stagger; /* > 0: each slot idles a seeded number of rounds in [0, start_stagger)
                            before its first game (benchmarks: spreads game ends over the
                            run); 0 = all games start in round 0 */
  int32_t engines_per_device; /* engines sharing this device (the CLI's numNNServerThreadsPerModel
                            engines on one GPU); with nn_batch_cap 0 a fused network's default
                            cap (one wave of network workgroups) is split between them, also
                            after a hot reload that changes the network path; 0 or 1 = alone */
} coffee_selfplay_config;

typedef struct coffee_selfplay coffee_selfplay;

typedef struct coffee_selfplay_stats {
  uint64_t rounds;          /* select -> NN -> backup rounds run */
  uint64_t playouts;        /* completed playouts (runSinglePlayout true) */
  uint64_t nn_evals;        /* network rows evaluated */
  uint64_t moves;           /* moves committed */
  uint64_t games_finished;
  uint64_t rows_written;    /* rows produced so far (drained + pending) */
  uint64_t rows_pending;    /* rows on the device not yet drained */
  uint64_t rows_dropped;    /* rows lost to a full row buffer (drain more often) */
  uint64_t games_dropped;   /* game records lost to a full record buffer (2 x num_games) */
  uint64_t errors;          /* device invariant violations (node pool exhausted, no move
                               candidate); nonzero makes stats return COFFEE_EINTERNAL */
  uint64_t tree_levels;     /* tree levels descended by all playouts (path nodes) */
  uint64_t tree_children;   /* children scanned at those path nodes (select reads each
                               path node and its k children; backup re-aggregates them) */
  uint64_t errors_node_pool; /* slots whose node pool ran out (part of errors) */
  uint64_t errors_edge_pool; /* slots whose edge pool (children past 16 per node) ran out */
  uint64_t edge_pool_peak;  /* largest edge-pool use of any slot so far (entries) */
  uint64_t edge_pool_cap;   /* edge-pool entries per slot and buffer */
  uint64_t nn_precision;    /* the precision the network runs (coffee_nn_precision; 0 = stand-in net) */
  /* Default precision on self-play's own positions: every 128th network launch of an engine
   * running the corrected instance re-evaluates its first 256 rows on the accurate one; the
   * largest |logit| difference is read at every stats / drain call and, past 2.5e-4, the
   * engine switches to the accurate instance for the rest of the run (the same model). */
  uint64_t nn_audits;         /* audited launches so far */
  uint64_t nn_audit_switches; /* switches to the accurate instance (0 or 1 per model) */
  double nn_audit_max_diff;   /* largest difference seen so far (0 before the first audit) */
} coffee_selfplay_stats;

int coffee_selfplay_create(const coffee_selfplay_config* cfg, coffee_selfplay** out);
/* Runs `rounds` rounds (one playout or root evaluation per game per round) on `stream`
 * (NULL = the engine's own stream).  Asynchronous: call coffee_selfplay_sync. */
int coffee_selfplay_step(coffee_selfplay* h, int rounds, void* stream);
int coffee_selfplay_sync(coffee_selfplay* h);
int coffee_selfplay_stats_get(coffee_selfplay* h, coffee_selfplay_stats* out);

/* Copies up to max_rows finished rows to HOST buffers and removes them from the device
 * buffer (trainingwrite.cpp:185-205 shapes; 5x5: pb = ceil(A/8) = 4):
 *   bin   [r][15][pb] u8   binaryInputNCHWPacked (big-endian bits, packBits :218-232)
 *   glob  [r][1]   f32     globalInputNC
 *   pol   [r][2][P] i16    policyTargetsNCMove
 *   gtgt  [r][64]  f32     globalTargetsNC
 *   value [r][5][A] i8     valueTargetsNCHW
 *   meta  [r][4]   i32     (slot, game number, turn, num moves) — not part of the .npz
 * Any output pointer may be NULL.  *n_out = rows copied. */
int coffee_selfplay_drain_rows(coffee_selfplay* h, int max_rows, uint8_t* bin, float* glob, int16_t* pol,
                               float* gtgt, int8_t* value, int32_t* meta, int* n_out);
/* Copies up to max_games finished-game records to HOST buffers and removes them
 * (the moves the reference's SGF writer prints, sgf.cpp:1526-1700 / selfplaymanager.cpp:350):
 *   header [g][4] i32  (slot, game number, number of moves, winner 0 draw / 1 black / 2 white)
 *   moves  [g][A][2] u8 (cell = y*x_len + x, direction 0..3 = N, W, NW, NE; 0xFF past the end)
 * Either output pointer may be NULL.  *n_out = records copied. */
int coffee_selfplay_drain_games(coffee_selfplay* h, int max_games, int32_t* header, uint8_t* moves, int* n_out);
/* Device-resident row hand-off for multi-GPU writers (the RCCL gather of SURVEY 8e;
 * trainingwrite.cpp:774-937 writes the rows afterwards).  Enqueued on the engine's own
 * stream, returns at once: every pending row is packed into dst (DEVICE memory,
 * [max_rows][coffee_row_bytes] u8, one record per row = bin, glob, pol, gtgt, value,
 * meta of coffee_selfplay_drain_rows back to back; max_rows >= the engine's row
 * capacity), the number of rows is copied to *count (HOST memory, pinned for an
 * asynchronous copy; valid once the engine stream has passed this call: wait on an
 * event recorded on coffee_selfplay_stream) and the engine's row buffer is emptied.
 * flags COFFEE_STAGE_DISCARD_GAMES: also drop the finished-game records (a caller that
 * writes no SGF).  The next steps may be enqueued before the rows are consumed. */
#define COFFEE_STAGE_DISCARD_GAMES 1
int coffee_selfplay_stage_rows(coffee_selfplay* h, void* dst, int max_rows, uint64_t* count, int flags);
int coffee_selfplay_row_capacity(coffee_selfplay* h, int* rows);
int coffee_row_bytes(int x, int y, int* bytes);
/* The engine's HIP stream (hipStream_t), for callers that order their own work
 * (events, copies, collectives) against the engine's. */
int coffee_selfplay_stream(coffee_selfplay* h, void** stream);
/* Replaces the network for every subsequent round of every game (the reference's
 * model hot reload with switchNetsMidGame, selfplay.cpp:135-260, play.cpp:1210-1226).
 * On error (unreadable / mismatched model) the current network stays in use. */
int coffee_selfplay_set_model(coffee_selfplay* h, const char* model_path);
/* The same from a CFNN file image in HOST memory (bytes long): a multi-rank host
 * broadcasts the new weights from rank 0 (RCCL) and every rank switches from the
 * received image, instead of each rank re-reading the file. */
int coffee_selfplay_set_model_bytes(coffee_selfplay* h, const void* data, uint64_t bytes);
int coffee_selfplay_destroy(coffee_selfplay* h);

/* Writes n rows (HOST arrays, drain_rows layout) as a training .npz in the reference's
 * format (TrainingWriteBuffers::writeToZipFile trainingwrite.cpp:566-587): members
 * binaryInputNCHWPacked, globalInputNC, policyTargetsNCMove, globalTargetsNC,
 * valueTargetsNCHW, each a v1.0 .npy with a 256-byte header; written to path.tmp
 * and renamed into place. */
int coffee_write_npz(const char* path, int n, int x, int y, const uint8_t* bin, const float* glob,
                     const int16_t* pol, const float* gtgt, const int8_t* value);

/* Device-side inspection for parity tests and tools (host outputs). */
/* info[16] i64: phase, rootK, nodeCount, rootIdx, gameNum, turn, pla, finished, winner,
 *               playouts, nnEvals, moves, gamesFinished, lastCell, lastDir, rng counter */
int coffee_selfplay_game_info(coffee_selfplay* h, int slot, int64_t* info);
/* Canonical tree of one game: nodes in breadth-first order from the root following
 * child slots in order (index-independent).  Per node 16 f32/u32 words, see DESIGN.md. */
int coffee_selfplay_game_tree(coffee_selfplay* h, int slot, int max_nodes, uint32_t* nodes, uint32_t* edges,
                              int* n_nodes);
/* The root's noised policy [P] (after temperature + Dirichlet). */
int coffee_selfplay_root_policy(coffee_selfplay* h, int slot, float* out);

/* Debug: the Student-t(3) CDF table the search uses (2000 f32). */
int coffee_debug_cdf_table(int x, int y, int win_len, float* out /* host */);
/* Debug: the Zobrist tables by cell (host): board [A][3][2], board2 [A][4][2],
 * player [3][2], init [2] (size-X ^ size-Y hashes), game_over [2]. */
int coffee_debug_zobrist(int x, int y, int win_len, uint64_t* board, uint64_t* board2, uint64_t* player,
                         uint64_t* init, uint64_t* game_over);

/* Kernel timing (HIP events on the engine stream) for roofline reporting:
 * which: 0 select, 1 network, 2 backup, 3 commit (+ rows), 4 backup + the next
 * round's select in one kernel (every round not followed by a commit, with the fast
 * fused network or the stand-in; the environment's COFFEE_FUSED_ROUNDS=0 / 1 at
 * creation: never / always).  Summed ms and launch count of the timed launches.  enable = 0 off, N > 0: every N-th launch of each
 * group is bracketed by an event pair (each pair costs a few microseconds of stream
 * gap, so N > 1 keeps a timed run representative of an untimed one). */
int coffee_selfplay_enable_timing(coffee_selfplay* h, int enable);
int coffee_selfplay_kernel_time(coffee_selfplay* h, int which, double* ms, uint64_t* launches);
/* Network evaluations performed by the timed network launches (sum of their batch sizes). */
int coffee_selfplay_timed_nn_evals(coffee_selfplay* h, uint64_t* evals);

#ifdef __cplusplus
}
#endif

#endif /* KATACOFFEE_H */
