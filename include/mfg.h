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

#define MFG_ABI_VERSION 1

#define MFG_MAX_AGENTS 64
#define MFG_MAX_ACTIONS 16
#define MFG_MAX_LAYERS 32
#define MFG_MAX_COMBINED 72
#define MFG_MAX_RULES 32
#define MFG_MAX_DOORS 64

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
  MFG_RULE_BATTERY_DECHARGE,     /* batteries/rules.py:9-87: f[0]=per_action_cost f[1]=discharge_reward i[0]=paralyze */
  MFG_RULE_DONE_BATTERY,         /* batteries/rules.py:90-128: as DECHARGE + i[1]=mode_single f[2]=reward_done */
  MFG_RULE_DONE_MAXSTEPS,        /* rules.py:202-225: i[0]=max_steps */
  MFG_RULE_RESPAWN_DIRT,         /* clean_up/rules.py:28-59: i[0]=freq i[1]=respawn_n f[0]=respawn_amount */
  MFG_RULE_SMEAR_DIRT,           /* clean_up/rules.py:62-86: dead (Q1), kept for rule order */
  MFG_RULE_DONE_DIRT,            /* clean_up/rules.py:10-25: f[0]=reward */
  MFG_RULE_DEST_REACH,           /* destinations/rules.py:20-54: f[0]=reward */
  MFG_RULE_DONE_DEST,            /* destinations/rules.py:57-92: f[0]=reach reward f[1]=reward_at_done i[0]=condition */
  MFG_RULE_MOVE_MAINTAINERS,     /* maintenance/rules.py:9-21 */
  MFG_RULE_DONE_MAINT_COLLISION  /* maintenance/rules.py:24-40 */
};

enum { MFG_DEST_ANY = 0, MFG_DEST_ALL = 1, MFG_DEST_SIMULTANEOUS = 2 };

typedef struct mfg_action {
  int32_t op, arg;
  double valid_reward, fail_reward;
  double aux0, aux1; /* ItemAction: valid / failed drop-off reward */
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
  const int32_t* floor_cells;    /* initial floor-list order: argwhere(level != '#') row-major (level_parser.py:467) */
  int32_t n_walls;
  const int32_t* wall_cells;     /* Wall u_int order (row-major argwhere '#') */
  int32_t n_doors;
  const int32_t* door_cells;     /* Door u_int order (row-major argwhere 'D') */
  int32_t door_closed_on_init, door_auto_close;
  int32_t pomdp_r;
  int32_t n_rays;
  const int32_t* ray_off;        /* [n_rays+1] prefix offsets into ray_pts (in points) */
  const int32_t* ray_pts;        /* [points][2] (dx, dy) from the ray origin, Bresenham order (ray_caster.py:141-199) */
  int32_t n_agents;
  int32_t agent_blocking[MFG_MAX_AGENTS];
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
  int32_t individual_rewards;
  uint32_t env_seed;
} mfg_spec;

/* Per env-step event record: everything the reference's info dict is built from (results.py:42-84,
 * factory.py:222-259). The host rebuilds the exact dict from (actions, events, spec). */
typedef struct mfg_events {
  uint8_t act[MFG_MAX_AGENTS];       /* bit0 action valid, bit1 action_introduced_collision,
                                        bit2 ItemAction took the drop-off branch, bit7 acted */
  uint8_t watch[MFG_MAX_AGENTS];     /* bit0 WatchCollisions result, bit1 battery discharged at post-step,
                                        bit2 DoneAtMaintainerCollision result for this agent */
  uint64_t door_coll;                /* doors that received a WatchCollisions result */
  uint64_t maint_coll;               /* maintainers that received a WatchCollisions result */
  int32_t respawn_items_value;       /* RespawnItems result value, -1 = no result this step */
  int32_t dirt_spawn_value;          /* RespawnDirt result value, -1 = no result */
  int32_t dirt_spawn_valid;
  int32_t dest_reach_agent[4];       /* agent index credited by DestinationReachReward per destination, -1 none */
  int32_t door_autoclose;            /* DoorAutoClose emitted its result */
  int32_t done_mask;                 /* bit r: rule r produced a VALID DoneResult */
  int32_t crashed;                   /* reference crash path hit (Q17): env flagged, done */
  int32_t step;
  int32_t maint_base;                /* u_int of the first maintainer (names 'Maintainer[maint_base + k]') */
} mfg_events;

/* ---- engine ABI (HIP) ---- */
typedef struct mfg_engine mfg_engine;

/* ABI version of the loaded library (== MFG_ABI_VERSION). */
int mfg_abi_version(void);

/* Create B = n_envs environments of `spec` on HIP device `device`. Replaces Factory.__init__
 * (factory.py:81-129) for a whole batch; no env is initialised until mfg_reset(init=1). */
int mfg_create(const mfg_spec* spec, int device, int64_t n_envs, mfg_engine** out);
int mfg_destroy(mfg_engine* e);
const char* mfg_last_error(void);

/* Reset envs (mask[b] != 0, or all if mask == NULL); Factory.reset (factory.py:134-148).
 * init = 0: reset existing envs. init & MFG_INIT_CREATE: first create the envs (Factory.__init__,
 * factory.py:81-129): env b is seeded like `random.seed(seed_base + b)` before `Factory(cfg)` (SURVEY
 * §8c seeding contract), or, with MFG_INIT_KEEP_MT, keeps the MT19937 state + index already imported
 * into its record (mfg_import_state), e.g. the caller's Python `random` state. MFG_INIT_NO_RESET stops
 * after creation (the reference's constructor does not reset). obs (device, may be NULL):
 * [B][A][lmax][d][d], obs_dtype 0 = float32, 1 = float64. */
enum { MFG_INIT_CREATE = 1, MFG_INIT_KEEP_MT = 2, MFG_INIT_NO_RESET = 4 };
int mfg_reset(mfg_engine* e, const uint8_t* mask, void* obs, int obs_dtype, int init, uint64_t seed_base,
              void* stream);

/* K fused env-steps of every env; Factory.step (factory.py:189-220) + auto-reset.
 * actions: device int32 [K][B][A] indices into each agent's action list, or NULL for synthetic uniform
 * actions from Philox4x32-10 keyed (philox_seed, env_base + b) at counter (step_base + k, agent).
 * Outputs (device, each may be NULL): reward f64 [K][B][A], done u8 [K][B], obs [K][B][A][lmax][d][d],
 * ev_act / ev_watch u8 [K][B][A] and ev_misc i32 [K][B][10] (the info-dict event record).
 * auto_reset != 0: an env whose step is done is reset before its obs row is rendered, so the row is the
 * new episode's first observation. Per step the engine launches k_logic, k_resetdone (auto_reset) and
 * k_obs (obs != NULL); pending floor-shuffle debt is replayed (mfg_replay) once before returning. */
int mfg_step(mfg_engine* e, int K, const int32_t* actions, uint32_t philox_seed, uint32_t env_base,
             int64_t step_base, double* reward, uint8_t* done, void* obs, int obs_dtype, uint8_t* ev_act,
             uint8_t* ev_watch, int32_t* ev_misc, int auto_reset, void* stream);

/* Replay pending membership-only floor shuffles (check_pos_validity, states.py:259-270, Q3). */
int mfg_replay(mfg_engine* e, void* stream);

/* Per-env state record layout (offsets) for host-side decoding; returns the number of ints written. */
int mfg_layout(const mfg_engine* e, int32_t* out);
void* mfg_state_ptr(mfg_engine* e);
int64_t mfg_state_bytes(const mfg_engine* e);
/* Per-kernel timing (HIP events recorded around every launch on the launch stream while enabled).
 * Kernel ids: MFG_K_LOGIC, MFG_K_RESETDONE, MFG_K_OBS, MFG_K_REPLAY, MFG_K_RESET.
 * mfg_profile_read synchronises on the last event, writes total milliseconds and launch counts per
 * kernel id (n entries, up to MFG_K_COUNT) and clears the accumulators. */
enum { MFG_K_LOGIC = 0, MFG_K_RESETDONE = 1, MFG_K_OBS = 2, MFG_K_REPLAY = 3, MFG_K_RESET = 4, MFG_K_COUNT = 5 };
int mfg_profile(mfg_engine* e, int enable);
int mfg_profile_read(mfg_engine* e, double* total_ms, int64_t* launches, int n);
/* Snapshots (checkpoint / resume, parity fixtures): whole state buffer device <-> device. */
int mfg_export_state(mfg_engine* e, void* dst, void* stream);
int mfg_import_state(mfg_engine* e, const void* src, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MFG_H_ */
