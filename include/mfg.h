/*
 * mfg.h — C-ABI of the MI355X batched step engine for the marl-factory-grid world.
 *
 * Drop-in boundary: this ABI replaces the per-object Python step of the reference
 *   Factory.step()            marl_factory_grid/environment/factory.py:189-220
 *   Gamestate.tick/check_done marl_factory_grid/utils/states.py:170-226
 *   StepRules hook fan-out    marl_factory_grid/utils/states.py:13-77
 *   Factory.reset()           marl_factory_grid/environment/factory.py:134-148
 *   OBSBuilder.build_for_all  marl_factory_grid/utils/observation_builder.py:96-103,138-235
 * The reference has no FFI of its own (pure Python); the Python host (mfg_amd.BatchedFactory /
 * mfg_amd.Factory) binds these symbols with ctypes.
 *
 * Conventions: plain C types only; all device buffers are caller-owned HIP device pointers
 * (e.g. torch data_ptr()); every call is stream-ordered on the given hipStream_t (passed as void*);
 * return 0 on success, <0 on error (mfg_last_error() describes it). No exceptions or exits cross the ABI.
 */
#ifndef MFG_H_
#define MFG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFG_ABI_VERSION 5

#define MFG_MAX_AGENTS 128  /* agents > 64: two 64-lane passes per agent-parallel step (mfg_kernels.h NW) */
#define MFG_MAX_ACTIONS 32
#define MFG_MAX_LAYERS 64  /* one lane per layer in the render */
#define MFG_MAX_COMBINED 144  /* members of one Combined layer: every other agent (Other) + the entity tags */
#define MFG_MAX_RULES 32
#define MFG_MAX_DOORS 128   /* doors > 64: the same two-pass kernels (the reference large_qquad level has 65) */
#define MFG_MAX_POSITIONS 64  /* configured spawn / destination cells per agent */

/* ---- action opcodes (reference: environment/actions.py, modules/<m>/actions.py) ---- */
enum {
  MFG_ACT_NOOP = 0,      /* actions.py:417-423 */
  MFG_ACT_MOVE = 1,      /* actions.py:426-455, arg = direction index (MFG_DIR_*) */
  MFG_ACT_CHARGE = 2,    /* modules/batteries/actions.py:11-31 */
  MFG_ACT_CLEAN = 3,     /* modules/clean_up/actions.py:11-36 */
  MFG_ACT_DEST = 4,      /* modules/destinations/actions.py:9-24 (crashes on a destination, Q17) */
  MFG_ACT_DOORUSE = 5,   /* modules/doors/actions.py:9-34 */
  MFG_ACT_ITEM = 6,      /* modules/items/actions.py:10-63 */
  MFG_ACT_MACHINE = 7    /* modules/machines/actions.py:10-25 */
};

/* Directions in the order of the reference's action classes North..NorthWest (helpers.py:36-42). */
enum { MFG_DIR_N = 0, MFG_DIR_NE, MFG_DIR_E, MFG_DIR_SE, MFG_DIR_S, MFG_DIR_SW, MFG_DIR_W, MFG_DIR_NW };

/* ---- observation tags (entity obs_tag, environment/entity/entity.py:386-392) ---- */
enum {
  MFG_TAG_WALLS = 0, MFG_TAG_DOORS, MFG_TAG_ITEMS, MFG_TAG_PODS, MFG_TAG_DROPOFFS, MFG_TAG_DIRT,
  MFG_TAG_DESTS, MFG_TAG_MACHINES, MFG_TAG_MAINTAINERS,
  MFG_TAG_AGENT0 = 16 /* + agent index: per-agent layer 'Agent[name]' */
};

/* ---- observation layer kinds (observation_builder.py:164-220) ---- */
enum {
  MFG_LAYER_ZERO = 0,     /* Placeholder / Inventory / positional group with no visible entity */
  MFG_LAYER_TAG = 1,      /* entities with obs_tag == tag placed relative to the agent */
  MFG_LAYER_COMBINED = 2, /* sum of the agent's Combined member tags (groups/utils.py:10-37) */
  MFG_LAYER_BATTERY = 3,  /* regex-bound Battery: flat[0] = charge of the first bound battery (Q11) */
  MFG_LAYER_GLOBALPOS = 4 /* regex-bound GlobalPosition: flat[0:2] = pos / level_shape (Q11) */
};

/* ---- rule opcodes, executed in spec order (config_parser.py:201-274, factory.py:117-119) ---- */
enum {
  MFG_RULE_SPAWN_BATTERIES = 1,  /* rules.py:145-167 + batteries/groups.py:33-39 */
  MFG_RULE_SPAWN_PODS,           /* i[0]=quantity i[1]=ignore_blocking */
  MFG_RULE_SPAWN_DROPOFFS,       /* i[0]=quantity i[1]=ignore_blocking */
  MFG_RULE_SPAWN_INVENTORIES,    /* items/groups.py:133-138 */
  MFG_RULE_SPAWN_ITEMS,          /* i[0]=quantity i[1]=ignore_blocking, items/groups.py:34-45 */
  MFG_RULE_SPAWN_DIRT,           /* clean_up/groups.py:70-95 (params in spec.dirt_*) */
  MFG_RULE_SPAWN_DESTS,          /* i[0]=quantity i[1]=ignore_blocking */
  MFG_RULE_SPAWN_MACHINES,       /* i[0]=quantity i[1]=ignore_blocking */
  MFG_RULE_SPAWN_MAINTAINERS,    /* i[0]=quantity i[1]=ignore_blocking */
  MFG_RULE_SPAWN_GLOBALPOS,      /* groups/utils.py:359-366 */
  MFG_RULE_DOOR_AUTOCLOSE,       /* doors/rules.py:8-28 */
  MFG_RULE_RESPAWN_ITEMS,        /* items/rules.py:9-43: i[0]=n_items i[1]=respawn_freq */
  MFG_RULE_WATCH_COLLISIONS,     /* rules.py:256-325: f[0]=reward i[0]=done_at_collisions f[1]=reward_at_done */
  MFG_RULE_BATTERY_DECHARGE,     /* batteries/rules.py:9-87: f[0]=per_action_cost f[1]=discharge_reward i[0]=paralyze
                                    i[2]=per-action cost dict (mfg_action.battery_cost), f[3]=its 'Noop' entry (paralyzed
                                    agents), i[3]=the dict has 'Noop' */
  MFG_RULE_DONE_BATTERY,         /* batteries/rules.py:90-128: as DECHARGE + i[1]=mode_single f[2]=reward_done */
  MFG_RULE_DONE_MAXSTEPS,        /* rules.py:202-225: i[0]=max_steps */
  MFG_RULE_RESPAWN_DIRT,         /* clean_up/rules.py:28-59: i[0]=freq i[1]=respawn_n f[0]=respawn_amount */
  MFG_RULE_SMEAR_DIRT,           /* clean_up/rules.py:62-86: dead (Q1), kept for rule order */
  MFG_RULE_DONE_DIRT,            /* clean_up/rules.py:10-25: f[0]=reward */
  MFG_RULE_DEST_REACH,           /* destinations/rules.py:20-54: f[0]=reward */
  MFG_RULE_DONE_DEST,            /* destinations/rules.py:57-92: f[0]=reach reward f[1]=reward_at_done i[0]=condition */
  MFG_RULE_MOVE_MAINTAINERS,     /* maintenance/rules.py:9-21 */
  MFG_RULE_DONE_MAINT_COLLISION, /* maintenance/rules.py:24-40 */
  MFG_RULE_SPAWN_DEST_ON_AGENT,  /* destinations/rules.py:136-162: one destination bound to each agent, on its cell */
  MFG_RULE_SPAWN_DEST_PER_AGENT, /* destinations/rules.py:95-133: spec.dest_entry_* (one bound destination per entry) */
  MFG_RULE_RANDOM_INIT_STEPS     /* rules.py:328-355 DoRandomInitialSteps (on_reset_post_spawn): i[0] = random_steps */
};

enum { MFG_DEST_ANY = 0, MFG_DEST_ALL = 1, MFG_DEST_SIMULTANEOUS = 2 };

typedef struct mfg_action {
  int32_t op, arg;
  double valid_reward, fail_reward;
  double aux0, aux1; /* ItemAction: valid / failed drop-off reward */
  double battery_cost; /* per-action battery cost of a BatteryDecharge rule whose per_action_costs is a dict
                          (rule i[2] = 1), keyed by the action's class name; NaN = key missing (KeyError) */
} mfg_action;

typedef struct mfg_layer {
  int32_t kind, tag;
} mfg_layer;

typedef struct mfg_rule {
  int32_t op;
  int32_t i[6];
  double f[6];
} mfg_rule;

/* Compiled environment specification (host: mfg_amd/spec.py compiles the reference YAML into this). */
typedef struct mfg_spec {
  int32_t abi_version;
  int32_t H, W;
  const uint8_t* level;          /* [H*W]: 0 floor, 1 wall, 2 door */
  int32_t n_floor;
  const int32_t* floor_cells;    /* initial floor-list order: argwhere(level != '#') row-major (level_parser.py:71) */
  int32_t n_walls;
  const int32_t* wall_cells;     /* Wall u_int order (row-major argwhere '#') */
  int32_t n_doors;
  const int32_t* door_cells;     /* Door u_int order (row-major argwhere 'D') */
  int32_t door_closed_on_init, door_auto_close;
  int32_t pomdp_r;               /* 0 = full observability: the window is the whole level (H x W), absolute cells,
                                    rays of radius min(H, W) (observation_builder.py:51,154-158) */
  int32_t n_rays;
  const int32_t* ray_off;        /* [n_rays+1] prefix offsets into ray_pts (in points) */
  const int32_t* ray_pts;        /* [points][2] (dx, dy) from the ray origin, Bresenham order (ray_caster.py:141-199) */
  int32_t n_agents;
  int32_t agent_blocking[MFG_MAX_AGENTS];
  int32_t n_positions[MFG_MAX_AGENTS];                      /* Agents.<name>.Positions (config_parser.py:181) */
  int32_t positions[MFG_MAX_AGENTS][MFG_MAX_POSITIONS];     /* cells; SpawnAgents takes the first empty one (rules.py:187-196) */
  int32_t n_actions[MFG_MAX_AGENTS];
  mfg_action actions[MFG_MAX_AGENTS][MFG_MAX_ACTIONS];
  int32_t n_layers[MFG_MAX_AGENTS];
  mfg_layer layers[MFG_MAX_AGENTS][MFG_MAX_LAYERS];
  int32_t combined_n[MFG_MAX_AGENTS];
  int32_t combined_tags[MFG_MAX_AGENTS][MFG_MAX_COMBINED];
  /* group parameters */
  int32_t has_batteries;  double battery_initial;           /* Batteries(initial_charge_level) */
  int32_t has_inventories;
  int32_t has_items;
  int32_t items_quantity;                                   /* Items coords_or_quantity */
  int32_t has_pods;       double pod_charge_rate;
  int32_t has_dropoffs;
  int32_t has_dirt;
  int32_t dirt_quantity;
  double dirt_initial_amount, dirt_clean_amount, dirt_max_global, dirt_max_local, dirt_amount_var, dirt_n_var;
  int32_t has_dests;      int32_t dest_action_counts;
  int32_t has_machines;   int32_t machine_work, machine_pause;
  int32_t has_maintainers;
  int32_t has_globalpos;
  int32_t has_doors;
  int32_t n_rules;
  mfg_rule rules[MFG_MAX_RULES];
  /* SpawnDestinationsPerAgent entries in YAML order: the agent, a coordinate list (q = 0) or a quantity q > 0 */
  int32_t n_dest_entries;
  int32_t dest_entry_agent[MFG_MAX_AGENTS];
  int32_t dest_entry_q[MFG_MAX_AGENTS];
  int32_t dest_entry_n[MFG_MAX_AGENTS];
  int32_t dest_entry_cells[MFG_MAX_AGENTS][MFG_MAX_POSITIONS];
  int32_t individual_rewards;
  uint32_t env_seed;
} mfg_spec;

/* ---- per env-step event rows written by mfg_step (the info dict is rebuilt from them) ----
 * ev_act   u8 [K][B][A]: bit0 action valid, bit1 action_introduced_collision (results.py:62-84),
 *                        bit2 ItemAction took the drop-off branch (items/actions.py:43-52), bit7 the agent acted
 * ev_watch u8 [K][B][A]: bit0 WatchCollisions result (rules.py:276-307), bit1 battery discharged at post-step
 *                        (batteries/rules.py:66-87), bit2 DoneAtMaintainerCollision result (maintenance/rules.py:32-40),
 *                        bits3..7 number of destinations this agent was credited with by the reach rule
 *                        (destinations/rules.py:34-54; TickResult entity = the agent)
 * ev_misc i32 [K][B][MFG_EV_MISC_N]: slots MFG_EVM_* below. */
#define MFG_EV_MISC_N 16
enum {
  MFG_EVM_DOOR_COLL_LO = 0,  /* doors (bit d) that received a WatchCollisions result, bits 0..31 */
  MFG_EVM_DOOR_COLL_HI = 1,  /* ... doors 32..63 (doors 64..127: MFG_EVM_DOOR_COLL_2 / _3) */
  MFG_EVM_RESPAWN_ITEMS = 2, /* RespawnItems result value, -1 = no result this step (items/rules.py:35-43) */
  MFG_EVM_DIRT_SPAWN = 3,    /* RespawnDirt result value, -1 = no result (clean_up/rules.py:49-59) */
  MFG_EVM_DIRT_VALID = 4,    /* ... and its validity */
  MFG_EVM_DEST_REACHED = 5,  /* destinations marked reached this step (sum of ev_watch bits 3..7) */
  MFG_EVM_FLAGS = 6,         /* bit0 DoorAutoClose emitted its result, bit1 crashed, bits 8..15 crash reason (MFG_CRASH_*) */
  MFG_EVM_DONE_MASK = 7,     /* bit r: rule r produced a VALID DoneResult; bit 31: WatchCollisions done */
  MFG_EVM_STEP = 8,          /* Gamestate.curr_step after the step (the info dict's 'step') */
  MFG_EVM_EPISODE = 9,       /* resets done so far */
  MFG_EVM_MAINT_COLL = 10,   /* maintainers (collection slot bit) that received a WatchCollisions result, slots 0..31 */
  MFG_EVM_MAINT_BASE = 11,   /* u_int of the first maintainer: names are 'Maintainer[base + slot]' */
  MFG_EVM_DOOR_COLL_2 = 12,  /* doors 64..95 that received a WatchCollisions result */
  MFG_EVM_DOOR_COLL_3 = 13,  /* doors 96..127 */
  MFG_EVM_MAINT_COLL_HI = 14,/* maintainer slots 32..63 */
  MFG_EVM_RESERVED = 15      /* 0 */
};

/* Crash reasons (reference crash paths; engine capacity). A crashed env reports done = 1. */
enum {
  MFG_CRASH_NONE = 0,
  MFG_CRASH_RULE = 1,        /* DestAction on a destination (AttributeError, Q17) or the RespawnItems TypeError (Q9) */
  MFG_CRASH_ROUTE = 2,       /* maintainer route: NodeNotFound / NetworkXNoPath */
  MFG_CRASH_NO_FREE = 3,     /* maintainer random_free_position on a full level (IndexError) */
  MFG_CRASH_NEXT_EMPTY = 4,  /* maintainer pops from an empty target list */
  MFG_CRASH_PATH_EMPTY = 5,  /* maintainer reads self._path[0] of an empty path */
  MFG_CRASH_MOVE = 6,        /* maintainer step not in MOVEMAP */
  MFG_CRASH_CAPACITY = 7,    /* engine capacity exceeded (dirt slots, id-pair list, reach counter) */
  MFG_CRASH_ACTION = 8       /* action index outside [0, n_actions[a]) (IndexError upstream, factory.py:201-206) */
};

/* Decoded form of one env-step's event rows (host side; the oracle reports the same record). */
typedef struct mfg_events {
  uint8_t act[MFG_MAX_AGENTS];       /* ev_act row */
  uint8_t watch[MFG_MAX_AGENTS];     /* ev_watch row */
  uint64_t door_coll;                /* doors 0..63: MFG_EVM_DOOR_COLL_LO | HI << 32 */
  uint64_t door_coll_hi;             /* doors 64..127: MFG_EVM_DOOR_COLL_2 | _3 << 32 */
  uint64_t maint_coll;               /* MFG_EVM_MAINT_COLL | MFG_EVM_MAINT_COLL_HI << 32 */
  int32_t respawn_items_value;       /* MFG_EVM_RESPAWN_ITEMS */
  int32_t dirt_spawn_value;          /* MFG_EVM_DIRT_SPAWN */
  int32_t dirt_spawn_valid;          /* MFG_EVM_DIRT_VALID */
  int32_t dest_reached;              /* MFG_EVM_DEST_REACHED */
  int32_t door_autoclose;            /* MFG_EVM_FLAGS bit0 */
  int32_t done_mask;                 /* MFG_EVM_DONE_MASK */
  int32_t crashed;                   /* MFG_EVM_FLAGS bit1 */
  int32_t crash_reason;              /* MFG_EVM_FLAGS bits 8..15 */
  int32_t step;                      /* MFG_EVM_STEP */
  int32_t episode;                   /* MFG_EVM_EPISODE */
  int32_t maint_base;                /* MFG_EVM_MAINT_BASE */
} mfg_events;

/* Decode one env's rows (ev_act/ev_watch: n_agents bytes, ev_misc: MFG_EV_MISC_N ints, all host memory). */
int mfg_decode_events(const uint8_t* ev_act, const uint8_t* ev_watch, const int32_t* ev_misc, int n_agents,
                      mfg_events* out);

/* ---- observation output modes (the obs_dtype argument of mfg_reset / mfg_step) ---- */
enum { MFG_OBS_F32 = 0, MFG_OBS_F64 = 1, MFG_OBS_PACKED = 2 };
#define MFG_MAX_EMB 128

/* Packed observations + fused policy-input projection. With obs_dtype MFG_OBS_PACKED the
 * `obs` argument is a HOST pointer to this descriptor; its device buffers are the k = 0 rows and the engine
 * offsets them per fused step. Per agent row (the dense row [lmax][h][w] of MFG_OBS_F32, whose values are
 * the reference's f64 obs cast like `observations.float()` in algorithms/marl/networks.py:52):
 *   count[a]       number of nonzero entries of the dense row (may exceed cap: only cap are stored)
 *   idx/val[a][i]  the nonzero entries, i < min(count, cap): flat index l*h*w + cell and the value, in
 *                  (64-cell block, layer, cell) order, i.e. ascending idx (the dense row's own order) when
 *                  h*w <= 64 or the observation rays have 9..12 points (pomdp_r 4 or 5) or more than 64 (the
 *                  long-ray render); slots >= count are
 *                  written as idx 0 / val 0, so a fixed-width gather over all cap slots is exact
 *   emb[a][j]      bias[j] + sum over ALL nonzero entries of val * wt[idx][j] (f32 fma in entry order): the
 *                  reference RecurrentAC.obs_proj (networks.py:19,52) evaluated without materialising the
 *                  dense row. wt = obs_proj.weight transposed, [lmax*h*w][emb_dim] row-major.
 * Any of idx/val (both or neither), count and emb may be NULL; emb needs wt and 0 < emb_dim <= MFG_MAX_EMB (128).
 * lmax*h*w must be < 65536 (u16 idx). */
typedef struct mfg_packed_obs {
  int32_t cap;        /* entries stored per agent row */
  int32_t emb_dim;    /* E; 0 = no projection */
  uint16_t* idx;      /* [K][B][A][cap] */
  float* val;         /* [K][B][A][cap] */
  int32_t* count;     /* [K][B][A] */
  const float* wt;    /* [lmax*h*w][E] */
  const float* bias;  /* [E] or NULL (zeros) */
  float* emb;         /* [K][B][A][E] */
} mfg_packed_obs;

/* ---- engine ABI (HIP) ---- */
typedef struct mfg_engine mfg_engine;

/* ABI version of the loaded library (== MFG_ABI_VERSION). */
int mfg_abi_version(void);

/* Create B = n_envs environments of `spec` on HIP device `device`. Replaces Factory.__init__
 * (factory.py:81-129) for a whole batch; no env is initialised until mfg_reset(init=1). Every bounded spec
 * count is validated (returns < 0 instead of reading out of bounds). The caller's current HIP device is
 * restored before any entry point returns; the engine's calls always run on `device`. */
int mfg_create(const mfg_spec* spec, int device, int64_t n_envs, mfg_engine** out);
/* Test-only: mfg_create with exact alternative code paths forced, so the parity tests can pin paths the
 * shipped configs never select (every field 0 = mfg_create's own choice). Results are identical either way. */
typedef struct mfg_variant {
  int32_t shuffle_table_path; /* 1: the shuffle blocks' table path (as if the exchange-order probe failed) */
  int32_t full_temper;        /* 1: the replay's full MT temper (levels with >= 16384 floor cells) */
  int32_t bfs_hbm;            /* 1: the maintainer BFS scratch in the per-env HBM pool (the grid128 layout) */
  int32_t pairs_lds;          /* > 0: at most this many identifier pairs in LDS, the rest in the HBM spill */
  int32_t render_slots;       /* > 0: at most this many resident waves in the long-ray render (k_obs_lr), so each
                                 strides over several envs */
  int32_t serial;             /* 1: every kernel on the caller's stream in launch order (no resets or replay on the
                                 engine's second stream beside the render): per-kernel times for attribution */
} mfg_variant;
int mfg_create_variant(const mfg_spec* spec, int device, int64_t n_envs, const mfg_variant* variant,
                       mfg_engine** out);
int mfg_destroy(mfg_engine* e);
/* Message of the last failed call on engine e (per engine); e == NULL: the calling thread's last failed
 * mfg_create / argument check. Valid until the next call on the same engine (or thread). */
const char* mfg_last_error(const mfg_engine* e);

/* Reset envs (mask[b] != 0, or all if mask == NULL); Factory.reset (factory.py:134-148).
 * init = 0: reset existing envs. init & MFG_INIT_CREATE: first create the envs (Factory.__init__,
 * factory.py:81-129): env b is seeded like `random.seed(seed_base + b)` before `Factory(cfg)` (SURVEY
 * §8c seeding contract), or, with MFG_INIT_KEEP_MT, keeps the MT19937 state + index already imported
 * into its record (mfg_import_state), e.g. the caller's Python `random` state. MFG_INIT_NO_RESET stops
 * after creation (the reference's constructor does not reset). obs (device, may be NULL):
 * [B][A][lmax][d][d], obs_dtype 0 = float32, 1 = float64; or MFG_OBS_PACKED with obs -> mfg_packed_obs. */
enum { MFG_INIT_CREATE = 1, MFG_INIT_KEEP_MT = 2, MFG_INIT_NO_RESET = 4 };
int mfg_reset(mfg_engine* e, const uint8_t* mask, void* obs, int obs_dtype, int init, uint64_t seed_base,
              void* stream);

/* K fused env-steps of every env; Factory.step (factory.py:189-220) + auto-reset.
 * actions: device int32 [K][B][A] indices into each agent's action list, or NULL for synthetic uniform
 * actions from Philox4x32-10 keyed (philox_seed, env_base + b) at counter (step_base + k, agent).
 * Outputs (device, each may be NULL): reward f64 [K][B][A], done u8 [K][B], obs [K][B][A][lmax][h][w]
 * (h = w = 2 pomdp_r + 1, or the level's H x W when pomdp_r == 0) in obs_dtype MFG_OBS_F32 / MFG_OBS_F64, or
 * the packed rows + fused projection of an mfg_packed_obs descriptor (obs_dtype MFG_OBS_PACKED; obs = host pointer),
 * ev_act / ev_watch u8 [K][B][A] and
 * ev_misc i32 [K][B][MFG_EV_MISC_N] (the info-dict event rows above).
 * An action index outside [0, n_actions[a]) crashes that env (MFG_CRASH_ACTION, done = 1).
 * flags (any other bit set: the call fails and nothing runs): MFG_STEP_AUTO_RESET: an env whose step is done is reset before its obs row is rendered, so
 * the row is the new episode's first observation. Per step the engine launches k_logic, k_resetdone (auto_reset)
 * and k_obs (obs != NULL); pending floor-shuffle debt is replayed (mfg_replay) once before returning (every step
 * on specs with long resets and an in-step floor-order consumer). MFG_STEP_DEFER_REPLAY: that final replay is
 * left to a later call (mfg_replay, or an mfg_step without the flag), e.g. once per learner window; results are
 * identical (the debt is always paid before the floor order or MT state is consumed), but the records' MT state
 * and floor order are not the reference's until it runs. Work on the engine's second stream is joined back to
 * `stream` before the call returns. */
enum { MFG_STEP_AUTO_RESET = 1, MFG_STEP_DEFER_REPLAY = 2 };
int mfg_step(mfg_engine* e, int K, const int32_t* actions, uint32_t philox_seed, uint32_t env_base,
             int64_t step_base, double* reward, uint8_t* done, void* obs, int obs_dtype, uint8_t* ev_act,
             uint8_t* ev_watch, int32_t* ev_misc, int flags, void* stream);

/* Replay pending membership-only floor shuffles (check_pos_validity, states.py:259-270, Q3). */
int mfg_replay(mfg_engine* e, void* stream);

/* Per-env state record layout (offsets) for host-side decoding, then the engine's launch facts (LDS slices,
 * o_logic, reset_overlap: 1 when a step's resets and their render run on the engine's second stream beside the
 * render of the other envs); returns the number of ints written (<= 64). */
int mfg_layout(const mfg_engine* e, int32_t* out);
void* mfg_state_ptr(mfg_engine* e);
int64_t mfg_state_bytes(const mfg_engine* e);
/* Per-kernel timing (HIP events recorded around every launch on the launch stream while enabled).
 * Kernel ids: MFG_K_LOGIC, MFG_K_RESETDONE, MFG_K_OBS, MFG_K_REPLAY, MFG_K_RESET, MFG_K_OBS_DONE (the render of
 * the envs reset in a step, on the engine's second stream; mfg_step with auto_reset and obs), MFG_K_REPLAY_SEL (the
 * debt of envs whose RespawnDirt fires in the coming step, paid before k_logic).
 * mfg_profile_read synchronises on the last event, writes total milliseconds and launch counts per
 * kernel id (n entries, up to MFG_K_COUNT) and clears the accumulators. */
enum { MFG_K_LOGIC = 0, MFG_K_RESETDONE = 1, MFG_K_OBS = 2, MFG_K_REPLAY = 3, MFG_K_RESET = 4, MFG_K_OBS_DONE = 5,
       MFG_K_REPLAY_SEL = 6, MFG_K_COUNT = 7 };
int mfg_profile(mfg_engine* e, int enable);
int mfg_profile_read(mfg_engine* e, double* total_ms, int64_t* launches, int n);
/* Snapshots (checkpoint / resume, parity fixtures): whole state buffer device <-> device. */
int mfg_export_state(mfg_engine* e, void* dst, void* stream);
int mfg_import_state(mfg_engine* e, const void* src, void* stream);

/* Measurement helper (not part of the Factory.step boundary): copy nbytes (a multiple of 16, 16-B aligned device
 * pointers) on the current device with a 16-B-per-lane streaming kernel, on `stream`. bench.py times it to report
 * the measured HBM peak beside the 8 TB/s spec figure. */
int mfg_hbm_copy(void* dst, const void* src, int64_t nbytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MFG_H_ */
