// mfg_device.h — device-side data structures of the MI355X batched step engine.
//
// Execution model: ONE WAVEFRONT PER ENVIRONMENT. A 64-lane wave owns one env for a whole launch:
//  * per-env entity tables are lane-distributed (lane i holds entity slot i of each group);
//  * the sequential parts of the reference step (agents act in list order, states.py:187-196) run as
//    wave-uniform control flow; set queries ("is there an X at cell c") are wave ballots;
//  * the RNG streams (MT19937 + floor-list permutation) live in the wave's LDS slice, the MT twist is
//    lane-parallel, rejection sampling for random.shuffle is resolved 64 draws at a time with ballots,
//    only the Fisher-Yates swap chain itself is serial;
//  * the observation render maps lanes to rays (walk) and then to window cells (placement), so obs
//    stores are coalesced runs of d*d values per layer.
// The env state lives in HBM as one contiguous record per env (layout below), so a wave's loads and
// stores of its env are contiguous/coalesced.
#pragma once
#include <stdint.h>

#include "../../include/mfg.h"

#define MFG_WAVE 64
#define MFG_HDR_N 40

// header slots (int32) of the per-env record
enum {
  H_STEP = 0,      // Gamestate.curr_step
  H_EPISODE,       // number of resets done
  H_CRASHED,       // reference crash path hit
  H_FROZEN,        // episode-1 agent objects replaced (Q11/Q12)
  H_OBS_INIT,      // OBSBuilder has built once (ray casters exist)
  H_DEBT,          // pending floor-list shuffles (replayed before any order-dependent consumer)
  H_MT_IDX,        // MT19937 index
  H_N_ITEMS, H_N_PODS, H_N_DROPS, H_N_DIRT, H_N_DESTS,
  H_ITEM_BASE, H_POD_BASE, H_DROP_BASE, H_DEST_BASE, H_BAT_BASE,
  H_ARRIVAL,       // Agents-group insertion counter (arrival order per cell)
  H_DONE,          // last step's done flag (auto-reset bookkeeping)
  H_OVERFLOW,      // capacity overflow (dirt piles > MFG_DIRT_MAX etc.) -> env flagged
  H_CNT_AGENT, H_CNT_BATTERY, H_CNT_POD, H_CNT_DROP, H_CNT_ITEM, H_CNT_DIRT, H_CNT_DEST, H_CNT_MACHINE,
  H_CNT_MAINT, H_CNT_GP,
  H_TOTAL_STEPS,   // env-steps since creation (Philox counter)
  H_N_MACHINES, H_MACHINE_BASE, H_N_MAINTS, H_MAINT_BASE,
  H_GRAPH_BUILT,   // Gamestate.floortile_graph exists (built once per env lifetime, states.py:82-87)
  H_DIRT_TOUCH,    // step-local: this step changed a dirt table (0 in every written-back record)
  H__END
};
static_assert(H__END <= MFG_HDR_N, "header overflow");

#define MFG_DIRT_MAX 1024  // dirt-pile slots per env: MfgDevSpec::dirt_cap (<= this) is sized per spec

// shuffle-block tables in LDS (u32): [rank table 64][counter][pad 3][j-hash table 512 (table path only)]
#define MFG_STAB_HASH 512
#define MFG_STAB_CTR 64
#define MFG_STAB_PTAB 68
#define MFG_STAB_N (MFG_STAB_PTAB + MFG_STAB_HASH)

// packed entity words (int32): pos in bits 0..15 (0xFFFF = VALUE_NO_POS), flags above
#define EW_POS(w) ((w) & 0xFFFF)
#define EW_ALIVE 0x10000     // member of its collection (Collection._data)
#define EW_PRESENT 0x20000   // present in the global pos_dict (identifier-dedup may keep it out, Q14)
#define EW_REACHED 0x40000   // destination reached
#define EW_NOPOS 0xFFFF
// destination bound to an agent (Object.bind_to, entity/object.py:140-148): bits 20..27 = agent index + 1
#define EW_BOUND_SHIFT 20
#define EW_BOUND(w) ((((w) >> EW_BOUND_SHIFT) & 0xFF) - 1)
// door word: bit0 open, bits 8..15 time_to_close, bit16 present in the global pos_dict
#define DW_OPEN 1
#define DW_TTC(w) (((w) >> 8) & 0xFF)
#define DW_PRESENT 0x10000

struct MfgLayout {
  int32_t size;  // bytes per env record (multiple of 16)
  int32_t o_hdr, o_rule_ctr, o_agent_pos, o_agent_arr, o_agent_par, o_frozen_org, o_frozen_gp;
  int32_t o_door, o_items, o_pods, o_drops, o_dests, o_dirt_pos, o_dirt_id;
  int32_t o_battery, o_frozen_bat, o_dirt_amt, o_pcg, o_mt, o_perm;
  int32_t o_machines, o_maints;       // lean part: group tables (pos | flags words)
  int32_t o_mstate, o_mpath, o_grank; // after perm: maintainer state, paths (u16 cells), graph ranks (u16)
  int32_t o_logic;                    // end of the step prefix (k_logic stages [0, o_logic); 16-B aligned)
};
// per-maintainer state ints: [path_n, path_head, next_n, last_serviced, next[mmax + 1]]
enum { MS_PATH_N = 0, MS_PATH_HEAD, MS_NEXT_N, MS_LAST_SERVICED, MS_NEXT };

// One observation layer of one agent as k_obs places it: value = popc(tags & unit_tags) +
// popc(agents & agent_bits) (members that encode 1.0, each once), unless a flag asks for more.
enum { LR_DOOR = 1, LR_DIRT = 2, LR_MACHINE = 4, LR_BATTERY = 8, LR_GLOBALPOS = 16, LR_ORDERED = 32 };
struct MfgLayerRec {
  uint32_t unit_tags;  // entity tags (< 16) counted as 1.0
  uint32_t flags;      // LR_*: door / dirt / machine value of a single-tag layer, regex-bound layers, or a
                       // Combined layer that needs its ordered left-to-right f64 sum (non-unit members)
  uint64_t agent_bits; // agents 0..63 counted as 1.0 (agents 64..127: MfgDevSpec::lrec_ab2)
};

struct MfgDevSpec {
  mfg_spec s;  // table pointers inside are HOST pointers: never dereferenced on the device
  // window: r = pomdp_r; oh x ow = (2r+1)^2 around the agent, or the whole level (r = 0, full observability,
  // observation_builder.py:51,154-158), dd = oh * ow cells. fr = ray radius = min(oh, ow) (Q13): the first-visit
  // table spans (2 fr + 1)^2 cells around the ray origin.
  int32_t HW, nf, nw, nd, A, r, oh, ow, dd, fr, nrays, maxpts, lmax;
  int32_t imax, pmax, dropmax, destmax;
  int32_t obs_agent_stride;  // lmax*dd
  const uint8_t* level;      // [HW] 0 floor 1 wall 2 door
  const uint8_t* door_of;    // [HW] door index or 0xFF
  const int32_t* wall_cells; // [nw]
  const int32_t* door_cells; // [nd]
  const int32_t* floor_init; // [nf]
  const int8_t* ray_pts;     // [nrays][maxpts][2] (dx, dy), padded
  const uint8_t* ray_len;    // [nrays]
  const uint64_t* ray_diag;  // [nrays] bit p: point p is a diagonal step from point p-1 (ray_caster.py:89-96)
  // [nf][nrays][3] per ray origin (floor index) and ray: the light-blocking bits of its points that depend
  // only on the static level (bit p: a wall at point p; a diagonal cut between two walls at step p), and
  // the points whose blocking depends on a door (recomputed from the cell map at render time). Null:
  // every point is tested at render time.
  const uint32_t* ray_static;
  int32_t n_wd_pairs;        // static identifier collisions Wall[k]/Door[k] that one ray fan can reach
  const int32_t* wd_pairs;   // [n_wd_pairs][3]: k, wall cell, door cell
  uint64_t pcg_init_hi, pcg_init_lo, pcg_inc_hi, pcg_inc_lo;  // default_rng(env_seed) state after seeding
  const uint16_t* base_map;  // [map_bytes / 2] static cell map of the obs render (CM_WALL bits), u16 cells
  const uint8_t* base_map8;  // [map_bytes8] the same with u8 cells (specs without machines/maintainers)
  int32_t map_bytes, map_bytes8;  // 2*HW / HW rounded up to 16
  int32_t step_rng;          // a rule consumes the floor order / RNG inside a step (dirt spawns)
  uint32_t respawn_mask;     // rule indices of RespawnDirt rules (k_replay_sel pays the debt of envs they fire in)
  MfgLayout L;
  int32_t lds_full;          // bytes of dynamic LDS per wave: full record + scratch + shuffle tables
  int32_t lds_logic;         // k_logic: lean record (o_mt bytes) or lds_full when step_rng
  int32_t lds_obs;           // k_obs: lean record + cell map + id-collision pairs + first-visit table + wall sup
  int32_t lds_obs_shared;    // the env-wide part of it (lean record, cell map, pairs; 16-B aligned)
  int32_t lds_obs_wave;      // the per-agent tables (multi-wave render: one copy per wave after the shared part)
  int32_t fv_words;          // first-visit table entries ((2d+1)^2, rounded up to 4)
  int32_t mmax, kmax;        // machines / maintainers per env (spawn quantities)
  int32_t mstate_ints, path_cap;  // ints per maintainer state; max stored path length (cells)
  int32_t bfs_off;           // offset of the BFS scratch in the full-record LDS slice (0 = none or in HBM)
  int32_t bfs_bytes;         // BFS scratch bytes per env (pred, succ, 2 fringes, level copy u16 + keys u32)
  uint8_t* bfs_pool;         // [B][bfs_bytes] BFS scratch in HBM when it does not fit the LDS slice, else null
  int32_t dirt_cap;          // dirt-pile slots per env record (spawn budget of one episode, multiple of 64)
  int32_t scratch_bytes;     // per-wave LDS scratch after the record (spawn positions + amounts, routes)
  int32_t max_pairs;         // capacity of the obs identifier-collision pair list (bounded by group sizes)
  int32_t pairs_lds;         // pairs held in the k_obs LDS slice; the rest go to pair_pool
  int32_t* pair_pool;        // [B][max_pairs - pairs_lds][3] HBM spill of the pair list, or null
  int32_t* rd_list;          // [2][B + 2]: per step parity, [0] = count, [2..] = envs k_logic flagged done (auto-reset)
  uint8_t* rd_flag;          // [B]: 1 if k_logic put the env on this step's done list (k_obs leaves it to the list render)
  const int16_t* cell_f;     // [HW] floor index of a cell, -1 for walls
  const uint8_t* node_ok;    // [nf] floor cell has a floor 8-neighbour (a node of points_to_graph)
  int32_t xchg_ordered;      // device applies conflicting ds_wrxchg lanes in lane order (probed at create)
  int32_t lds_replay_per_wave;  // k_replay slice: [hdr][MT + u16 perm image of the record][sink][tables]
  int32_t replay_mtperm, replay_sink_off, replay_stab_off, replay_stab_n;
  int32_t replay_top14;      // nf < 16384: shuffle draws use only the top 14 tempered bits (replay_shuffle_t)
  // Combined obs layers whose members all encode 1.0 (walls, items, pods, drop-offs, destinations,
  // maintainers, agents) and appear once: the left-to-right f64 sum of 0/1 terms equals the member count,
  // so k_obs places popc(tags & comb_unit_tags) + popc(agents & comb_agents) instead of a member loop
  int32_t comb_fast[MFG_MAX_AGENTS];
  uint32_t comb_unit_tags[MFG_MAX_AGENTS];
  uint64_t comb_agents[MFG_MAX_AGENTS];
  uint64_t comb_agents2[MFG_MAX_AGENTS];  // agents 64..127
  // 64-lane passes of the agent- and door-parallel code: 1, or 2 when the spec has more than 64 agents or doors (the
  // NW template parameter of k_logic / k_reset / k_resetdone; the render branches on the agent count at run time)
  int32_t lane_passes;
  const MfgLayerRec* lrec;   // [A][lmax] layer records
  const uint64_t* lrec_ab2;  // [A][lmax] the layer records' agents 64..127 counted as 1.0 (long-ray render only)
  // long-ray render (maxpts == 0: rays of 65..255 points, k_obs_lr): the ray table with 16-bit offsets, and the
  // per-agent tables (first-visit table, wall suppression, sinks, dirt bitmap, agent masks, dirt map, packed queue:
  // the same layout as the LDS render's per-wave part) of each resident render wave in HBM instead of LDS
  const uint32_t* ray_pts16; // [nrays][lrpts] (dx & 0xFFFF) | dy << 16 per point, padded; null unless maxpts == 0
  int32_t lrpts;             // points per ray slot of ray_pts16 (a multiple of 32)
  int32_t obs_slots;         // resident long-ray render waves (grid of k_obs_lr), each owning one pool slot
  int64_t obs_slot_bytes;    // bytes per slot
  uint8_t* obs_pool;         // [2][obs_slots][obs_slot_bytes]: slots of the all-env render, then of the done-list
                             // render (the two may run at the same time on the two streams of mfg_step)
  // rules that act in each step phase, in rule order (spawn rules and the like act only at reset)
  int32_t n_ph[3];                       // tick_step, tick_post_step, on_check_done
  uint8_t ph_rule[3][MFG_MAX_RULES];
};
