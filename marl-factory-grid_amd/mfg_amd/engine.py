"""ctypes binding of the HIP engine (libmfg_hip.so, C-ABI in include/mfg.h).

The product path is the HIP library: there is no CPU fallback. If the library is missing or no GPU is
visible the constructor raises. Device memory for inputs/outputs is owned by the caller (torch tensors);
the engine owns the per-env state records.
"""
import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import abi

LIB_PATH = Path(os.environ.get('MFG_HIP_LIB') or Path(__file__).resolve().parent / '_lib' / 'libmfg_hip.so')
EV_MISC = abi.EV_MISC_N  # MFG_EV_MISC_N (include/mfg.h)
HDR_N = 40  # MFG_HDR_N (csrc/mfg_device.h)
KERNELS = ['k_logic', 'k_resetdone', 'k_obs', 'k_replay', 'k_reset', 'k_obs_done', 'k_replay_sel']  # MFG_K_* ids (include/mfg.h)

LAYOUT_KEYS = ['size', 'o_hdr', 'o_rule_ctr', 'o_agent_pos', 'o_agent_arr', 'o_agent_par', 'o_frozen_org',
               'o_frozen_gp', 'o_door', 'o_items', 'o_pods', 'o_drops', 'o_dests', 'o_dirt_pos', 'o_dirt_id',
               'o_battery', 'o_frozen_bat', 'o_dirt_amt', 'o_pcg', 'o_mt', 'o_perm', 'lmax', 'obs_agent_stride',
               'lds_full', 'xchg_ordered', 'o_machines', 'o_maints', 'o_mstate', 'o_mpath', 'o_grank', 'dirt_cap',
               'lds_logic', 'lds_obs', 'lds_replay', 'bfs_off', 'bfs_bytes', 'max_pairs', 'scratch_bytes', 'o_logic',
               'reset_overlap']
# header slots (csrc/mfg_device.h)
HDR = {k: i for i, k in enumerate([
    'step', 'episode', 'crashed', 'frozen', 'obs_init', 'debt', 'mt_idx', 'n_items', 'n_pods', 'n_drops',
    'n_dirt', 'n_dests', 'item_base', 'pod_base', 'drop_base', 'dest_base', 'bat_base', 'arrival', 'done',
    'overflow', 'cnt_agent', 'cnt_battery', 'cnt_pod', 'cnt_drop', 'cnt_item', 'cnt_dirt', 'cnt_dest',
    'cnt_machine', 'cnt_maint', 'cnt_gp', 'total_steps', 'n_machines', 'machine_base', 'n_maints', 'maint_base',
    'graph_built', 'dirt_touch'])}

_lib = None


def load_lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f'HIP engine library missing: {LIB_PATH} (run __graft_entry__.build())')
    L = C.CDLL(str(LIB_PATH))
    L.mfg_create.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.POINTER(C.c_void_p)]
    L.mfg_create.restype = C.c_int
    L.mfg_create_variant.argtypes = [C.c_void_p, C.c_int, C.c_int64, C.c_void_p, C.POINTER(C.c_void_p)]
    L.mfg_create_variant.restype = C.c_int
    L.mfg_destroy.argtypes = [C.c_void_p]
    L.mfg_destroy.restype = C.c_int
    L.mfg_last_error.argtypes = [C.c_void_p]
    L.mfg_last_error.restype = C.c_char_p
    L.mfg_decode_events.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.mfg_decode_events.restype = C.c_int
    L.mfg_layout.argtypes = [C.c_void_p, C.c_void_p]
    L.mfg_layout.restype = C.c_int
    L.mfg_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_void_p]
    L.mfg_reset.restype = C.c_int
    L.mfg_step.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int64, C.c_void_p,
                           C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                           C.c_void_p]
    L.mfg_step.restype = C.c_int
    L.mfg_replay.argtypes = [C.c_void_p, C.c_void_p]
    L.mfg_replay.restype = C.c_int
    L.mfg_export_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.mfg_export_state.restype = C.c_int
    L.mfg_import_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.mfg_import_state.restype = C.c_int
    L.mfg_state_bytes.argtypes = [C.c_void_p]
    L.mfg_state_bytes.restype = C.c_int64
    L.mfg_profile.argtypes = [C.c_void_p, C.c_int]
    L.mfg_profile.restype = C.c_int
    L.mfg_profile_read.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L.mfg_profile_read.restype = C.c_int
    L.mfg_hbm_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    L.mfg_hbm_copy.restype = C.c_int
    L.mfg_abi_version.restype = C.c_int
    if L.mfg_abi_version() != abi.ABI_VERSION:
        raise RuntimeError('libmfg_hip.so ABI version mismatch')
    _lib = L
    return L


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def hbm_copy(dst, src, stream=None):
    """dst.copy_(src) through the library's 16-B-per-lane streaming kernel (mfg_hbm_copy; bench.py's measured HBM
    peak). Both contiguous device tensors of the same byte size on the current device."""
    import torch
    n = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == n and dst.is_contiguous() and src.is_contiguous()
    st = stream if stream is not None else torch.cuda.current_stream(src.device)
    _check(load_lib().mfg_hbm_copy(_ptr(dst), _ptr(src), n, C.c_void_p(st.cuda_stream)), 'mfg_hbm_copy')


def _check(rc, what, h=None):
    if rc != 0:
        raise RuntimeError(f'{what} failed: {load_lib().mfg_last_error(h).decode()}')


class MfgVariant(C.Structure):
    """include/mfg.h mfg_variant: exact alternative code paths forced for the parity tests."""
    _fields_ = [('shuffle_table_path', C.c_int32), ('full_temper', C.c_int32), ('bfs_hbm', C.c_int32),
                ('pairs_lds', C.c_int32), ('render_slots', C.c_int32),
                ('serial', C.c_int32)]


class Engine:
    """B environments of one compiled spec on one GPU. variant: test-only {field: value} of mfg_variant."""

    def __init__(self, spec, n_envs, device=0, variant=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError('mfg_amd.Engine needs a GPU (HIP); no CPU fallback exists')
        self.torch = torch
        self.L = load_lib()
        self.spec = spec
        self.B = int(n_envs)
        self.device = torch.device('cuda', device)
        torch.cuda.set_device(self.device)
        h = C.c_void_p()
        if variant:
            v = MfgVariant(**variant)
            _check(self.L.mfg_create_variant(C.byref(spec.c), device, self.B, C.byref(v), C.byref(h)),
                   'mfg_create_variant')
        else:
            _check(self.L.mfg_create(C.byref(spec.c), device, self.B, C.byref(h)), 'mfg_create')
        self.h = h
        lay = np.zeros(64, np.int32)
        n = self.L.mfg_layout(self.h, lay.ctypes.data_as(C.c_void_p))
        self.layout = dict(zip(LAYOUT_KEYS, [int(x) for x in lay[:n]]))
        self.lmax = self.layout['lmax']
        self.A = spec.n_agents
        self.d = spec.d
        self.obs_hw = tuple(spec.obs_hw)  # (d, d), or the level shape with full observability

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            self.L.mfg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def obs_shape(self, K=None):
        s = (self.B, self.A, self.lmax) + self.obs_hw
        return s if K is None else (K,) + s

    def _obs_arg(self, obs, K):
        """(pointer, obs_dtype) of a dense obs tensor or a PackedObs (MFG_OBS_PACKED: host descriptor)."""
        if isinstance(obs, PackedObs):
            if obs.engine is not self or obs.K < K:
                raise ValueError('PackedObs was made for another engine or fewer fused steps')
            return C.byref(obs.desc), abi.OBS_PACKED
        if obs is not None and not obs.is_contiguous():
            raise ValueError('obs must be contiguous')
        return _ptr(obs), (abi.OBS_F64 if (obs is not None and obs.dtype == self.torch.float64) else abi.OBS_F32)

    def reset(self, obs=None, mask=None, init=False, seed_base=0):
        op, dt = self._obs_arg(obs, 1)
        _check(self.L.mfg_reset(self.h, _ptr(mask), op, dt, int(init), int(seed_base), self._stream()),
               'mfg_reset', self.h)

    def step(self, K=1, actions=None, philox_seed=0, env_base=0, step_base=0, reward=None, done=None, obs=None,
             ev_act=None, ev_watch=None, ev_misc=None, auto_reset=True, defer_replay=False):
        op, dt = self._obs_arg(obs, K)
        _check(self.L.mfg_step(self.h, int(K), _ptr(actions), int(philox_seed) & 0xFFFFFFFF, int(env_base),
                               int(step_base), _ptr(reward), _ptr(done), op, dt, _ptr(ev_act),
                               _ptr(ev_watch), _ptr(ev_misc), int(bool(auto_reset)) | (2 if defer_replay else 0),
                               self._stream()), 'mfg_step',
               self.h)

    def profile(self, enable=True):
        """Record HIP events around every kernel launch (on the launch stream) while enabled."""
        _check(self.L.mfg_profile(self.h, int(bool(enable))), 'mfg_profile')

    def profile_read(self):
        """{kernel: (total_ms, launches)} since the last read (synchronises on the last event)."""
        n = len(KERNELS)
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int64)
        _check(self.L.mfg_profile_read(self.h, ms.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p), n),
               'mfg_profile_read')
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(KERNELS)}

    def export_state(self):
        t = self.torch.empty((self.B, self.layout['size']), dtype=self.torch.uint8, device=self.device)
        _check(self.L.mfg_export_state(self.h, _ptr(t), self._stream()), 'mfg_export_state')
        return t

    def import_state(self, t):
        assert t.dtype == self.torch.uint8 and t.numel() == self.B * self.layout['size']
        _check(self.L.mfg_import_state(self.h, _ptr(t.contiguous()), self._stream()), 'mfg_import_state')


class PackedObs:
    """Device buffers of the packed observation mode (MFG_OBS_PACKED, `mfg_packed_obs` in include/mfg.h) for
    K fused steps, SURVEY §8(f) f3. Per (step, env, agent) row of the dense obs [lmax, h, w]:

    * ``idx`` u16 / ``val`` f32 [K, B, A, cap]: the nonzero entries (flat index ``l*h*w + cell``, value as
      ``observations.float()`` in the reference network, algorithms/marl/networks.py:52); slots past the count
      are 0 / 0.0, so a fixed-width gather over all ``cap`` slots is exact;
    * ``count`` i32 [K, B, A]: the true number of nonzero entries (``> cap`` = truncated row, see ``check()``);
    * ``emb`` f32 [K, B, A, E]: ``bias + sum val * weight[:, idx]``, the reference ``RecurrentAC.obs_proj``
      (networks.py:19) fused into the render, over ALL nonzero entries.

    ``weight`` is an ``nn.Linear(lmax*h*w, E).weight`` ([E, lmax*h*w]); ``set_projection`` refreshes the
    engine's transposed copy after an optimizer step (same device pointers, no reallocation)."""

    def __init__(self, engine, K=1, cap=32, weight=None, bias=None, entries=True, count=True):
        torch = engine.torch
        self.engine, self.K, self.cap = engine, int(K), int(cap) if entries else 0
        B, A = engine.B, engine.A
        self.kdim = engine.lmax * engine.obs_hw[0] * engine.obs_hw[1]
        dev = engine.device
        self.idx = torch.zeros((K, B, A, self.cap), dtype=torch.uint16, device=dev) if entries else None
        self.val = torch.zeros((K, B, A, self.cap), dtype=torch.float32, device=dev) if entries else None
        self.count = torch.zeros((K, B, A), dtype=torch.int32, device=dev) if count else None
        self.E = 0
        self.wt = self.bias = self.emb = None
        if weight is not None:
            E = int(weight.shape[0])
            if not 0 < E <= abi.MAX_EMB or int(weight.shape[1]) != self.kdim:
                raise ValueError(f'projection weight must be [E <= {abi.MAX_EMB}, {self.kdim}]')
            self.E = E
            self.wt = torch.empty((self.kdim, E), dtype=torch.float32, device=dev)
            self.bias = torch.zeros(E, dtype=torch.float32, device=dev)
            self.emb = torch.zeros((K, B, A, E), dtype=torch.float32, device=dev)
            self.set_projection(weight, bias)
        self.desc = self._make_desc()

    def _make_desc(self):
        d = abi.MfgPackedObs()
        d.cap, d.emb_dim = self.cap, self.E
        for f in ('idx', 'val', 'count', 'wt', 'bias', 'emb'):
            t = getattr(self, f)
            setattr(d, f, t.data_ptr() if t is not None else None)
        return d

    def view(self, k):
        """Row k as a K = 1 PackedObs sharing this one's buffers (e.g. one slot of a rollout window)."""
        v = PackedObs.__new__(PackedObs)
        v.engine, v.K, v.cap, v.kdim, v.E = self.engine, 1, self.cap, self.kdim, self.E
        for f in ('idx', 'val', 'count', 'emb'):
            t = getattr(self, f)
            setattr(v, f, t[k:k + 1] if t is not None else None)
        v.wt, v.bias = self.wt, self.bias
        v.desc = v._make_desc()
        return v

    def set_projection(self, weight, bias=None):
        """Copy an nn.Linear weight [E, kdim] (and bias [E]) into the engine's transposed f32 buffers."""
        with self.engine.torch.no_grad():
            self.wt.copy_(weight.detach().t())
            if bias is None:
                self.bias.zero_()
            else:
                self.bias.copy_(bias.detach())

    def check(self):
        """Raise if a stored row was truncated (count > cap); one device->host sync."""
        if self.count is not None and self.cap and int(self.count.max()) > self.cap:
            raise RuntimeError(f'packed obs row has {int(self.count.max())} nonzero entries > cap {self.cap}')

    def dense(self, k=0):
        """Scatter row k back into a dense f32 obs [B, A, lmax, h, w] (test / debugging view)."""
        torch = self.engine.torch
        B, A = self.engine.B, self.engine.A
        out = torch.zeros((B, A, self.kdim), dtype=torch.float32, device=self.engine.device)
        out.scatter_add_(2, self.idx[k].long(), self.val[k])
        return out.view((B, A, self.engine.lmax) + self.engine.obs_hw)


class RecordView:
    """Host-side decoder of one env state record (numpy bytes), using the engine's layout."""

    def __init__(self, rec: np.ndarray, layout, spec):
        self.b = rec.tobytes() if isinstance(rec, np.ndarray) else bytes(rec)
        self.L = layout
        self.spec = spec

    def i32(self, off, n):
        return np.frombuffer(self.b, np.int32, n, off)

    def f64(self, off, n):
        return np.frombuffer(self.b, np.float64, n, off)

    def hdr(self, k):
        return int(self.i32(self.L['o_hdr'], HDR_N)[HDR[k]])

    def agent_pos(self):
        return self.i32(self.L['o_agent_pos'], self.spec.n_agents)

    def battery(self):
        return self.f64(self.L['o_battery'], self.spec.n_agents)

    def doors(self):
        w = self.i32(self.L['o_door'], self.spec.c.n_doors)
        return (w & 1), ((w >> 8) & 0xFF), ((w >> 16) & 1)

    def group(self, name):
        off, hn = {'items': ('o_items', 'n_items'), 'pods': ('o_pods', 'n_pods'), 'drops': ('o_drops', 'n_drops'),
                   'dests': ('o_dests', 'n_dests'), 'dirt': ('o_dirt_pos', 'n_dirt')}[name]
        return self.i32(self.L[off], self.hdr(hn))

    def dirt(self):
        n = self.hdr('n_dirt')
        return self.i32(self.L['o_dirt_pos'], n), self.i32(self.L['o_dirt_id'], n), self.f64(self.L['o_dirt_amt'], n)

    def mt(self):
        st = np.frombuffer(self.b, np.uint32, 624, self.L['o_mt']).copy()
        return np.concatenate([st, np.asarray([self.hdr('mt_idx')], np.uint32)])

    def perm(self):
        return np.frombuffer(self.b, np.uint16, self.spec.c.n_floor, self.L['o_perm']).astype(np.int32)

    def pcg(self):
        return np.frombuffer(self.b, np.uint64, 4, self.L['o_pcg'])


def events_from_rows(ev_act, ev_watch, ev_misc):
    """One env-step's device event rows -> dict with the mfg_events fields (include/mfg.h), decoded by the
    library's own mfg_decode_events so the host and the C-ABI share one row contract."""
    L = load_lib()
    act = np.ascontiguousarray(ev_act, np.uint8)
    watch = np.ascontiguousarray(ev_watch, np.uint8)
    misc = np.ascontiguousarray(ev_misc, np.int32)
    assert misc.size == abi.EV_MISC_N and act.size == watch.size
    ev = abi.MfgEvents()
    _check(L.mfg_decode_events(act.ctypes.data, watch.ctypes.data, misc.ctypes.data, int(act.size), C.byref(ev)),
           'mfg_decode_events')
    out = {k: getattr(ev, k) for k, _ in abi.MfgEvents._fields_}
    out['act'] = [int(x) for x in act]
    out['watch'] = [int(x) for x in watch]
    return out
