"""CPU: spec compiler behaviour and the C-ABI surface (library loads, every declared symbol exported,
struct layouts agree between include/mfg.h, the ctypes mirror and the compiled libraries)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def test_compile_headline_spec():
    from mfg_amd.spec import compile_spec
    s = compile_spec('large8.yaml')
    assert s.n_agents == 8 and s.H == 24 and s.W == 62
    assert len(s.floor_cells) == 1077 and len(s.door_cells) == 15 and len(s.wall_cells) == 411
    assert s.agent_names[1] == 'Wolfgang_the_0th' and s.agent_names[3] == 'Wolfgang_the_2nd'
    assert s.action_idents[0] == ['Noop', 'do_charge_action', 'use_door', 'ITEMACTION', 'north', 'east', 'south',
                                  'west', 'north_east', 'south_east', 'south_west', 'north_west']
    assert s.layer_names[0] == ['Combined(Agent[Wolfgang])', 'Battery', 'ChargePods', 'Doors', 'Items',
                                'Inventory', 'DropOffLocations']
    assert s.rule_names[-5:] == ['SpawnEntity(Batteries)', 'SpawnEntity(ChargePods)',
                                 'SpawnEntity(DropOffLocations)', 'SpawnEntity(Inventories)', 'SpawnEntity(Items)']


@pytest.mark.parametrize('cfg', ['large8.yaml', 'rooms4.yaml', 'simple1.yaml', 'alltest16.yaml'])
def test_named_action_space_matches_fixture(cfg):
    import golden_compare as G
    from mfg_amd.spec import compile_spec
    s = compile_spec(cfg)
    rec, _ = G.load(Path(cfg).stem, 0)
    got = {f'Agent[{n}]': {a: i for i, a in enumerate(s.action_idents[k])} for k, n in enumerate(s.agent_names)}
    assert got == rec['named_action_space']
    assert {f'Agent[{n}]': s.layer_names[k] for k, n in enumerate(s.agent_names)} == rec['obs_layers']


def test_unsupported_classes_are_rejected(tmp_path):
    from mfg_amd.spec import compile_spec, UnsupportedSpec
    bad = tmp_path / 'bad.yaml'
    bad.write_text("General: {env_seed: 69, individual_rewards: true, level_name: large, pomdp_r: 3}\n"
                   "Agents: {W: {Actions: [Noop, Teleport], Observations: [Walls]}}\n"
                   "Entities: {}\nRules: {}\n")
    with pytest.raises(UnsupportedSpec):
        compile_spec(bad)
    bad.write_text("General: {env_seed: 69, individual_rewards: true, level_name: large, pomdp_r: 3}\n"
                   "Agents: {W: {Actions: [Noop], Observations: [Walls]}}\n"
                   "Entities: {}\nRules: {Defaults: {}}\n")
    with pytest.raises(UnsupportedSpec):
        compile_spec(bad)
    # Q26: global (non-individual) rewards crash the reference's step; rejected, not silently mis-summed
    bad.write_text("General: {env_seed: 69, individual_rewards: false, level_name: large, pomdp_r: 3}\n"
                   "Agents: {W: {Actions: [Noop], Observations: [Walls]}}\n"
                   "Entities: {}\nRules: {}\n")
    with pytest.raises(UnsupportedSpec, match='individual_rewards'):
        compile_spec(bad)


def _header_functions():
    txt = ''.join(p.read_text() for p in sorted((ROOT / 'include').glob('*.h')))
    return sorted(set(re.findall(r'\b(mfg_[a-z_]+)\s*\(', txt)))


def test_hip_library_exports_every_declared_symbol():
    lib_path = ROOT / 'marl-factory-grid_amd' / 'mfg_amd' / '_lib' / 'libmfg_hip.so'
    if not lib_path.exists():
        import __graft_entry__
        __graft_entry__.build_hip()
    lib = C.CDLL(str(lib_path))  # loads without a GPU: no compute call is made here
    funcs = _header_functions()
    assert 'mfg_step' in funcs and 'mfg_create' in funcs
    for f in funcs:
        assert hasattr(lib, f), f'{f} declared in include/*.h but not exported'
    lib.mfg_abi_version.restype = C.c_int
    assert lib.mfg_abi_version() == 5


def _hip_lib():
    from mfg_amd.engine import LIB_PATH
    if not LIB_PATH.exists():
        import __graft_entry__
        __graft_entry__.build_hip()
    lib = C.CDLL(str(LIB_PATH))
    lib.mfg_last_error.argtypes = [C.c_void_p]
    lib.mfg_last_error.restype = C.c_char_p
    return lib


def _header_enum(prefix):
    txt = (ROOT / 'include' / 'mfg.h').read_text()
    out = {m.group(1): int(m.group(2)) for m in re.finditer(rf'\b({prefix}[A-Z0-9_]+)\s*=\s*(\d+)', txt)}
    out.update({m.group(1): int(m.group(2)) for m in re.finditer(rf'#define\s+({prefix}[A-Z0-9_]+)\s+(\d+)', txt)})
    return out


def test_event_row_contract_matches_header():
    """The ev_misc row width and slot numbers of include/mfg.h are the ones the host decodes with."""
    from mfg_amd import abi
    from mfg_amd.engine import EV_MISC
    h = _header_enum('MFG_EV')
    assert h['MFG_EV_MISC_N'] == abi.EV_MISC_N == EV_MISC == 16
    for k, v in h.items():
        if k.startswith('MFG_EVM_'):
            assert getattr(abi, k[4:]) == v, k
    crash = _header_enum('MFG_CRASH_')
    assert sorted(crash.values()) == sorted(abi.CRASH_NAMES)


def test_decode_events_through_the_abi():
    """mfg_decode_events (pure host code) decodes every slot of a row triple; events_from_rows uses it."""
    from mfg_amd import abi
    from mfg_amd.engine import events_from_rows
    A = 5
    act = np.array([0x81, 0x80, 0x83, 0, 0x85], np.uint8)
    watch = np.array([1 | (2 << 3), 2, 4, 0, 8], np.uint8)
    misc = np.zeros(abi.EV_MISC_N, np.int32)
    misc[abi.EVM_DOOR_COLL_LO] = -2147483647  # bit 0 and bit 31
    misc[abi.EVM_DOOR_COLL_HI] = 5
    misc[abi.EVM_RESPAWN_ITEMS] = -1
    misc[abi.EVM_DIRT_SPAWN] = 3
    misc[abi.EVM_DIRT_VALID] = 1
    misc[abi.EVM_DEST_REACHED] = 3
    misc[abi.EVM_FLAGS] = 1 | 2 | (8 << 8)
    misc[abi.EVM_DONE_MASK] = -2147483648 | 4
    misc[abi.EVM_STEP] = 17
    misc[abi.EVM_EPISODE] = 2
    misc[abi.EVM_MAINT_COLL] = 6
    misc[abi.EVM_MAINT_BASE] = 40
    misc[abi.EVM_DOOR_COLL_2] = 1 << 3  # door 67
    misc[abi.EVM_DOOR_COLL_3] = -2147483648  # door 127
    misc[abi.EVM_MAINT_COLL_HI] = 1  # maintainer slot 32
    ev = events_from_rows(act, watch, misc)
    assert ev['act'] == list(act) and ev['watch'] == list(watch)
    assert ev['door_coll'] == (1 | (1 << 31) | (5 << 32))
    assert ev['respawn_items_value'] == -1 and ev['dirt_spawn_value'] == 3 and ev['dirt_spawn_valid'] == 1
    assert ev['dest_reached'] == 3 and ev['door_autoclose'] == 1 and ev['crashed'] == 1
    assert ev['crash_reason'] == 8 and ev['done_mask'] == (-2147483648 | 4)
    assert ev['step'] == 17 and ev['episode'] == 2 and ev['maint_coll'] == (6 | (1 << 32)) and ev['maint_base'] == 40
    assert ev['door_coll_hi'] == (1 << 3) | (1 << 63)


def test_create_validates_spec_without_touching_the_gpu():
    """Out-of-range spec counts are refused by mfg_create before any HIP call, with a message
    from mfg_last_error(NULL)."""
    from mfg_amd.spec import compile_spec
    lib = _hip_lib()
    lib.mfg_create.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.POINTER(C.c_void_p)]
    cases = [('n_actions', lambda c: c.n_actions.__setitem__(0, 33), 'n_actions'),
             ('n_layers', lambda c: c.n_layers.__setitem__(1, 65), 'n_layers'),
             ('combined_n', lambda c: c.combined_n.__setitem__(0, 145), 'combined_n'),
             ('n_rules', lambda c: setattr(c, 'n_rules', 33), 'n_rules'),
             ('move arg', lambda c: setattr(c.actions[0][4], 'arg', 9), 'direction'),
             ('layer tag', lambda c: setattr(c.layers[0][2], 'tag', 99), 'tag'),
             ('abi', lambda c: setattr(c, 'abi_version', 1), 'ABI')]
    for name, mutate, msg in cases:
        spec = compile_spec('large8.yaml')
        mutate(spec.c)
        h = C.c_void_p()
        rc = lib.mfg_create(C.byref(spec.c), 0, 4, C.byref(h))
        assert rc < 0 and not h.value, name
        assert msg in lib.mfg_last_error(None).decode(), (name, lib.mfg_last_error(None))


def test_struct_layouts_agree():
    import oracle as O
    from mfg_amd import abi
    L = O.lib()
    L.oracle_sizeof_spec.restype = C.c_int
    L.oracle_sizeof_events.restype = C.c_int
    L.oracle_sizeof_res.restype = C.c_int
    assert C.sizeof(abi.MfgSpec) == L.oracle_sizeof_spec()
    assert C.sizeof(abi.MfgEvents) == L.oracle_sizeof_events()
    assert C.sizeof(O.Res) == L.oracle_sizeof_res()
    L.oracle_sizeof_packed_obs.restype = C.c_int
    assert C.sizeof(abi.MfgPackedObs) == L.oracle_sizeof_packed_obs()


def test_philox_known_answer():
    from philox import philox_u32
    # Random123 philox4x32-10 KAT: key 0, counter 0 -> first word 0x6627e8d5
    assert int(philox_u32(0, 0, 0, 0)) == 0x6627E8D5


@pytest.mark.parametrize('level,pomdp_r,pts_range', [('grid128', 31, (33, 64)), ('grid128', 32, (65, 66)),
                                                     ('large_qquad', 0, (33, 64)), ('grid128', 0, (129, 129)),
                                                     ('grid128', 126, (254, 254)), ('grid128', 127, None)])
def test_ray_length_limits(tmp_path, level, pomdp_r, pts_range):
    """Rays of 2 * pomdp_r + 2 points, or min(H, W) + 1 with full observability (Q13). Up to 64 points render from
    registers, 65..255 points on the long-ray render (k_obs_lr): pomdp_r <= 126 and full observability on levels with
    min(H, W) <= 254 compile (grid128 full: 129-point rays); longer rays are refused."""
    from mfg_amd.spec import compile_spec, UnsupportedSpec
    cfg = tmp_path / 'c.yaml'
    cfg.write_text(f"General: {{env_seed: 69, individual_rewards: true, level_name: {level}, pomdp_r: {pomdp_r}}}\n"
                   "Agents: {W: {Actions: [Noop, Move8], Observations: [Walls]}}\nEntities: {}\nRules: {}\n")
    if pts_range:
        spec = compile_spec(cfg)
        pts = max(int(b) - int(a) for a, b in zip(spec.c.ray_off[:spec.c.n_rays], spec.c.ray_off[1:spec.c.n_rays + 1]))
        assert pts_range[0] <= pts <= pts_range[1]
    else:
        with pytest.raises(UnsupportedSpec, match='255 points'):
            compile_spec(cfg)


@pytest.mark.parametrize('n_agents,extra_layers,n_noop,n_pos,error', [
    (40, 'Doors, ', 10, 20, None),            # wide40: 41 layers, 20 actions, 20 positions
    (63, '', 24, 64, None),                   # 64 layers ('Other' of 63 agents + Walls), 32 actions, 64 positions
    (64, 'Doors, ', 1, 1, 'too many observation layers'),
    (4, '', 25, 1, 'too many actions'),
    (4, '', 1, 65, 'positions')])
def test_capacity_limits(tmp_path, n_agents, extra_layers, n_noop, n_pos, error):
    """Round 5: up to 64 observation layers per agent (one lane per layer in the render), 32 actions and 64
    configured spawn positions per agent; past them the spec compiler refuses cleanly."""
    from mfg_amd.spec import compile_spec, UnsupportedSpec
    pos = ', '.join(f"'({8 + i // 60}, {1 + i % 60})'" for i in range(n_pos))
    acts = ', '.join(['Noop'] * n_noop + ['Move8'])
    cfg = tmp_path / 'c.yaml'
    cfg.write_text("General: {env_seed: 7, individual_rewards: true, level_name: large, pomdp_r: 2}\n"
                   f"Agents: {{A: {{Actions: [{acts}], Observations: [Walls, {extra_layers}Other], "
                   f"Positions: [{pos}], Clones: {n_agents - 1}}}}}\nEntities: {{Doors: }}\nRules: {{}}\n")
    if error is None:
        s = compile_spec(cfg)
        assert s.n_agents == n_agents and max(s.n_layers) == n_agents + (1 if extra_layers else 0)
        assert max(s.n_actions) == n_noop + 8 and len(s.agent_positions[0]) == n_pos
    else:
        with pytest.raises(UnsupportedSpec, match=error):
            compile_spec(cfg)


@pytest.mark.parametrize('n_agents,error', [(81, None), (128, None), (129, 'agents > 128')])
def test_agent_capacity(tmp_path, n_agents, error):
    """Round 6: up to 128 agents (two 64-lane passes in the agent-parallel kernels; a Combined layer holds every
    other agent), past that a clean refusal. The reference's Agents collection is positional and uncapped."""
    from mfg_amd.spec import compile_spec, UnsupportedSpec
    cfg = tmp_path / 'c.yaml'
    cfg.write_text("General: {env_seed: 7, individual_rewards: true, level_name: large_qquad, pomdp_r: 2}\n"
                   "Agents: {A: {Actions: [Noop, Move8, DoorUse], Observations: [{Combined: [Other, Walls]}, Doors], "
                   f"Clones: {n_agents - 1}}}}}\nEntities: {{Doors: }}\nRules: {{}}\n")
    if error is None:
        s = compile_spec(cfg)
        assert s.n_agents == n_agents and s.c.n_doors == 65 and max(s.n_layers) == 2
        assert s.c.combined_n[n_agents - 1] == n_agents  # the other agents + Walls
    else:
        with pytest.raises(UnsupportedSpec, match=error):
            compile_spec(cfg)


def test_large_qquad_with_its_doors_compiles():
    """VERDICT r5 missing 1: the reference's own large_qquad level keeps its 65 Doors (indices 0..64)."""
    from mfg_amd.spec import compile_spec
    s = compile_spec('qquad_doors.yaml')
    assert s.c.n_doors == 65 and s.c.has_doors


def test_record_header_slots_match_device_enum():
    """engine.HDR (the host decoder's header slot names) follows the device enum in csrc/mfg_device.h slot for slot,
    so RecordView reads the slot the kernels write (H_STEP .. H_DIRT_TOUCH); and both fit MFG_HDR_N."""
    import re
    from pathlib import Path
    from mfg_amd.engine import HDR, HDR_N
    src = (Path(__file__).resolve().parents[1] / 'marl-factory-grid_amd' / 'csrc' / 'mfg_device.h').read_text()
    body = src[src.index('H_STEP = 0'):src.index('H__END')]
    body = re.sub(r'//[^\n]*', '', body)
    names = [n.strip()[2:].lower() for n in body.replace('= 0', '').split(',') if n.strip()]
    assert names == list(HDR), (names, list(HDR))
    assert len(names) <= HDR_N == int(re.search(r'#define MFG_HDR_N (\d+)', src).group(1))
