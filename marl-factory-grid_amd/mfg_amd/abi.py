"""ctypes mirror of include/mfg.h (the engine's C-ABI). Field order and sizes must match the header exactly;
tests/test_abi.py checks sizeof() against the compiled libraries."""
import ctypes as C

MAX_AGENTS = 128
MAX_ACTIONS = 32
MAX_LAYERS = 64
MAX_COMBINED = 144
MAX_RULES = 32
MAX_DOORS = 128
MAX_POSITIONS = 64

# action opcodes
ACT_NOOP, ACT_MOVE, ACT_CHARGE, ACT_CLEAN, ACT_DEST, ACT_DOORUSE, ACT_ITEM, ACT_MACHINE = range(8)
# directions (North..NorthWest) and their (dx, dy) from utils/helpers.py:36-42
DIR_NAMES = ['North', 'NorthEast', 'East', 'SouthEast', 'South', 'SouthWest', 'West', 'NorthWest']
DIR_IDENT = ['north', 'north_east', 'east', 'south_east', 'south', 'south_west', 'west', 'north_west']
DIR_DELTA = [(-1, 0), (-1, 1), (0, 1), (1, 1), (1, 0), (1, -1), (0, -1), (-1, -1)]

# observation tags
TAG_WALLS, TAG_DOORS, TAG_ITEMS, TAG_PODS, TAG_DROPOFFS, TAG_DIRT, TAG_DESTS, TAG_MACHINES, TAG_MAINTAINERS = range(9)
TAG_AGENT0 = 16
# layer kinds
LAYER_ZERO, LAYER_TAG, LAYER_COMBINED, LAYER_BATTERY, LAYER_GLOBALPOS = range(5)

# rule opcodes
(RULE_SPAWN_BATTERIES, RULE_SPAWN_PODS, RULE_SPAWN_DROPOFFS, RULE_SPAWN_INVENTORIES, RULE_SPAWN_ITEMS,
 RULE_SPAWN_DIRT, RULE_SPAWN_DESTS, RULE_SPAWN_MACHINES, RULE_SPAWN_MAINTAINERS, RULE_SPAWN_GLOBALPOS,
 RULE_DOOR_AUTOCLOSE, RULE_RESPAWN_ITEMS, RULE_WATCH_COLLISIONS, RULE_BATTERY_DECHARGE, RULE_DONE_BATTERY,
 RULE_DONE_MAXSTEPS, RULE_RESPAWN_DIRT, RULE_SMEAR_DIRT, RULE_DONE_DIRT, RULE_DEST_REACH, RULE_DONE_DEST,
 RULE_MOVE_MAINTAINERS, RULE_DONE_MAINT_COLLISION, RULE_SPAWN_DEST_ON_AGENT, RULE_SPAWN_DEST_PER_AGENT,
 RULE_RANDOM_INIT_STEPS) = range(1, 27)

DEST_ANY, DEST_ALL, DEST_SIMULTANEOUS = range(3)

ABI_VERSION = 5
# ev_misc row (include/mfg.h MFG_EVM_*)
EV_MISC_N = 16
(EVM_DOOR_COLL_LO, EVM_DOOR_COLL_HI, EVM_RESPAWN_ITEMS, EVM_DIRT_SPAWN, EVM_DIRT_VALID, EVM_DEST_REACHED, EVM_FLAGS,
 EVM_DONE_MASK, EVM_STEP, EVM_EPISODE, EVM_MAINT_COLL, EVM_MAINT_BASE, EVM_DOOR_COLL_2, EVM_DOOR_COLL_3,
 EVM_MAINT_COLL_HI, EVM_RESERVED) = range(EV_MISC_N)
# the ev_misc column and bit of door d's / maintainer slot k's WatchCollisions result
EVM_DOOR_COLS = (EVM_DOOR_COLL_LO, EVM_DOOR_COLL_HI, EVM_DOOR_COLL_2, EVM_DOOR_COLL_3)
EVM_MAINT_COLS = (EVM_MAINT_COLL, EVM_MAINT_COLL_HI)
# crash reasons (MFG_CRASH_*)
CRASH_NAMES = {0: 'none', 1: 'reference crash path (DestAction on a destination Q17 / RespawnItems Q9)',
               2: 'maintainer route: no path', 3: 'maintainer: no free cell', 4: 'maintainer: empty target list',
               5: 'maintainer: empty path', 6: 'maintainer: step not in MOVEMAP', 7: 'engine capacity exceeded',
               8: 'action index out of range'}


class MfgAction(C.Structure):
    _fields_ = [('op', C.c_int32), ('arg', C.c_int32), ('valid_reward', C.c_double), ('fail_reward', C.c_double),
                ('aux0', C.c_double), ('aux1', C.c_double), ('battery_cost', C.c_double)]


class MfgLayer(C.Structure):
    _fields_ = [('kind', C.c_int32), ('tag', C.c_int32)]


class MfgRule(C.Structure):
    _fields_ = [('op', C.c_int32), ('i', C.c_int32 * 6), ('f', C.c_double * 6)]


class MfgSpec(C.Structure):
    _fields_ = [
        ('abi_version', C.c_int32),
        ('H', C.c_int32), ('W', C.c_int32),
        ('level', C.POINTER(C.c_uint8)),
        ('n_floor', C.c_int32), ('floor_cells', C.POINTER(C.c_int32)),
        ('n_walls', C.c_int32), ('wall_cells', C.POINTER(C.c_int32)),
        ('n_doors', C.c_int32), ('door_cells', C.POINTER(C.c_int32)),
        ('door_closed_on_init', C.c_int32), ('door_auto_close', C.c_int32),
        ('pomdp_r', C.c_int32),
        ('n_rays', C.c_int32), ('ray_off', C.POINTER(C.c_int32)), ('ray_pts', C.POINTER(C.c_int32)),
        ('n_agents', C.c_int32),
        ('agent_blocking', C.c_int32 * MAX_AGENTS),
        ('n_positions', C.c_int32 * MAX_AGENTS),
        ('positions', (C.c_int32 * MAX_POSITIONS) * MAX_AGENTS),
        ('n_actions', C.c_int32 * MAX_AGENTS),
        ('actions', (MfgAction * MAX_ACTIONS) * MAX_AGENTS),
        ('n_layers', C.c_int32 * MAX_AGENTS),
        ('layers', (MfgLayer * MAX_LAYERS) * MAX_AGENTS),
        ('combined_n', C.c_int32 * MAX_AGENTS),
        ('combined_tags', (C.c_int32 * MAX_COMBINED) * MAX_AGENTS),
        ('has_batteries', C.c_int32), ('battery_initial', C.c_double),
        ('has_inventories', C.c_int32),
        ('has_items', C.c_int32),
        ('items_quantity', C.c_int32),
        ('has_pods', C.c_int32), ('pod_charge_rate', C.c_double),
        ('has_dropoffs', C.c_int32),
        ('has_dirt', C.c_int32),
        ('dirt_quantity', C.c_int32),
        ('dirt_initial_amount', C.c_double), ('dirt_clean_amount', C.c_double), ('dirt_max_global', C.c_double),
        ('dirt_max_local', C.c_double), ('dirt_amount_var', C.c_double), ('dirt_n_var', C.c_double),
        ('has_dests', C.c_int32), ('dest_action_counts', C.c_int32),
        ('has_machines', C.c_int32), ('machine_work', C.c_int32), ('machine_pause', C.c_int32),
        ('has_maintainers', C.c_int32),
        ('has_globalpos', C.c_int32),
        ('has_doors', C.c_int32),
        ('n_rules', C.c_int32),
        ('rules', MfgRule * MAX_RULES),
        ('n_dest_entries', C.c_int32),
        ('dest_entry_agent', C.c_int32 * MAX_AGENTS),
        ('dest_entry_q', C.c_int32 * MAX_AGENTS),
        ('dest_entry_n', C.c_int32 * MAX_AGENTS),
        ('dest_entry_cells', (C.c_int32 * MAX_POSITIONS) * MAX_AGENTS),
        ('individual_rewards', C.c_int32),
        ('env_seed', C.c_uint32),
    ]


class MfgEvents(C.Structure):
    _fields_ = [
        ('act', C.c_uint8 * MAX_AGENTS),
        ('watch', C.c_uint8 * MAX_AGENTS),
        ('door_coll', C.c_uint64),
        ('door_coll_hi', C.c_uint64),
        ('maint_coll', C.c_uint64),
        ('respawn_items_value', C.c_int32),
        ('dirt_spawn_value', C.c_int32),
        ('dirt_spawn_valid', C.c_int32),
        ('dest_reached', C.c_int32),
        ('door_autoclose', C.c_int32),
        ('done_mask', C.c_int32),
        ('crashed', C.c_int32),
        ('crash_reason', C.c_int32),
        ('step', C.c_int32),
        ('episode', C.c_int32),
        ('maint_base', C.c_int32),
    ]


# observation output modes (include/mfg.h MFG_OBS_*) and the packed-obs descriptor
OBS_F32, OBS_F64, OBS_PACKED = range(3)
MAX_EMB = 128


class MfgPackedObs(C.Structure):
    _fields_ = [
        ('cap', C.c_int32),
        ('emb_dim', C.c_int32),
        ('idx', C.c_void_p),
        ('val', C.c_void_p),
        ('count', C.c_void_p),
        ('wt', C.c_void_p),
        ('bias', C.c_void_p),
        ('emb', C.c_void_p),
    ]
