"""On-GPU MARL training over the batched engine: packed observations gathered straight
into the policy input, rollouts and A2C updates without a host round trip.

Reference anchors:
  * the network: ``algorithms/marl/networks.py:7-69`` ``RecurrentAC`` (same constructor, parameter names and
    layers, so its ``state_dict`` loads either way);
  * the loss: ``algorithms/marl/base_ac.py:185-226`` ``compute_advantages`` / ``actor_critic`` / ``learn``
    (RMSprop lr 3e-4 eps 1e-5, ``clip_grad_norm_(0.5)``, ``base_ac.py:45-47,219-225``);
  * the loop: ``base_ac.py:90-150`` ``train_loop`` (act on ``(obs, last_action, hidden)``, learn every
    ``n_steps``), batched over B envs x A agents, one shared network (``snac.py:8-33``).

What is different from the reference, and why:
  * The obs never exist densely. The engine renders each agent's row as packed nonzero entries plus the fused
    projection ``obs_proj(obs.float())`` (``mfg_packed_obs``, include/mfg.h); acting reads that projection,
    learning re-evaluates ``obs_proj`` on the stored entries with ``F.embedding_bag`` (the same sum over the
    nonzero terms, differentiable in the weight). C3 moves ~6 B x 32 entries per agent row instead of
    1,372 B of dense f32.
  * The memory is aligned: entry t holds (o_t, a_{t-1}) as the network input and a_t, r_t, d_t as targets.
    ``train_loop`` stores the obs of the step *before* each action (``base_ac.py:119``), so its loss pairs
    a_t with o_{t-1}; the loss function itself (``actor_critic``) is used unchanged and is pinned by a
    fixture produced by the reference (tests/golden/marl_a2c.npz, tools/gen_golden_marl.py).
  * Episodes end per env (auto-reset): an entry whose previous step was done starts a new episode, so its
    action input is -1 (padding) and the recurrent state restarts from zero, as the reference does at every
    ``env.reset()`` (``base_ac.py:98-100``). The reference's GRU runs the window in one ``nn.GRU`` call; here
    too: every row's episode segments become sequences of one packed batch (``_Segments``), so a restart
    inside the window costs no extra launches. Acting (one step) uses the fused ``torch.gru_cell``.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical


SPLIT_ROWS = 2048  # rows per split of a tall-K weight-gradient GEMM (_tall_tn)


def _tall_tn(a, b, rows=None):
    """a^T @ b for tall a [K, m], b [K, n] (weight gradients over N*T rows: K ~ 393K, m x n ~ 100 x 100). As one
    GEMM the library tiles only the small m x n output (a handful of workgroups walking all of K: ~1 ms each on the
    MI355X at C3's learner); split into K / rows batched GEMMs (one workgroup set per split) and summed it fills the
    chip. Same products, different summation order (fp32 rounding only)."""
    rows = rows or SPLIT_ROWS
    k = a.shape[0]
    s = k // rows
    if s < 2:
        return a.t() @ b
    k0 = s * rows
    # (the split sum as a ones-row GEMM instead measured slower: 4.60M vs 4.83M env-steps/s in the A2C loop)
    out = torch.bmm(a[:k0].reshape(s, rows, -1).transpose(1, 2), b[:k0].reshape(s, rows, -1)).sum(0)
    if k0 < k:
        out = out + a[k0:].t() @ b[k0:]
    return out


class _Linear(torch.autograd.Function):
    """x @ w^T + b on [M, in] rows with the weight gradient by _tall_tn (nn.Linear's backward is one tall-K GEMM)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return g @ w, _tall_tn(g, x), g.sum(0)


def _lin(mod, x):
    """mod (nn.Linear) applied to x [..., in] through _Linear (same parameters)."""
    lead = x.shape[:-1]
    return _Linear.apply(x.reshape(-1, x.shape[-1]), mod.weight, mod.bias).view(*lead, -1)


class _Embed(torch.autograd.Function):
    """nn.Embedding lookup whose weight gradient is onehot(idx)^T @ g by _tall_tn: the embedding's own backward
    scatters M rows onto a table of ~10 rows (action embedding), serialised on the few hot rows."""

    @staticmethod
    def forward(ctx, idx, w, padding_idx):
        ctx.save_for_backward(idx)
        ctx.n, ctx.pad = w.shape[0], padding_idx
        return w[idx]

    @staticmethod
    def backward(ctx, g):
        idx, = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        oh = F.one_hot(idx.reshape(-1), ctx.n).to(g2.dtype)
        gw = _tall_tn(oh, g2)
        if ctx.pad is not None:
            gw[ctx.pad] = 0  # nn.Embedding(padding_idx): that row gets no gradient
        return None, gw, None


class RecurrentAC(nn.Module):
    """``algorithms/marl/networks.py:7-69`` with the same parameters; adds the packed-obs projection and a
    step-wise recurrent pass with episode restarts."""

    def __init__(self, observation_size, n_actions, obs_emb_size, action_emb_size, hidden_size_actor,
                 hidden_size_critic, n_agents, use_agent_embedding=True, gru_window='fused'):
        super().__init__()
        # how a window of T > 1 steps runs the GRUs: 'fused' = _GRUWindow (both GRUs, the window's GEMMs batched,
        # forward and backward written out), 'cells' = torch.gru_cell (one fused kernel) per step and GRU under
        # autograd, 'segments' = one nn.GRU call over packed episode segments (_Segments). Measured on the MI355X
        # (C3, B = 8,192, n_steps 5): 'cells' 32.7 vs 'segments' 102.3 ms per update (MIOpen's packed-sequence GRU)
        if gru_window not in ('fused', 'cells', 'segments'):
            raise ValueError("gru_window must be 'fused', 'cells' or 'segments'")
        self.gru_window = gru_window
        observation_size = int(np.prod(observation_size))
        self.n_layers = 1
        self.n_actions = n_actions
        self.use_agent_embedding = use_agent_embedding
        self.hidden_size_actor = hidden_size_actor
        self.hidden_size_critic = hidden_size_critic
        self.action_emb_size = action_emb_size
        self.obs_proj = nn.Linear(observation_size, obs_emb_size)
        self.action_emb = nn.Embedding(n_actions + 1, action_emb_size, padding_idx=0)
        self.agent_emb = nn.Embedding(n_agents, action_emb_size)
        # networks.py:22 sizes the mix input as obs + n_agents * action_emb with the agent embedding (only
        # consistent for n_agents == 2); kept so reference checkpoints load
        mix_in_size = obs_emb_size + action_emb_size if not use_agent_embedding else \
            obs_emb_size + n_agents * action_emb_size
        self.mix = nn.Sequential(nn.Tanh(), nn.Linear(mix_in_size, obs_emb_size), nn.Tanh(),
                                 nn.Linear(obs_emb_size, obs_emb_size))
        self.gru_actor = nn.GRU(obs_emb_size, hidden_size_actor, batch_first=True, num_layers=self.n_layers)
        self.gru_critic = nn.GRU(obs_emb_size, hidden_size_critic, batch_first=True, num_layers=self.n_layers)
        self.action_head = nn.Sequential(nn.Linear(hidden_size_actor, hidden_size_actor), nn.Tanh(),
                                         nn.Linear(hidden_size_actor, n_actions))
        self.critic_head = nn.Sequential(nn.Linear(hidden_size_critic, hidden_size_critic), nn.Tanh(),
                                         nn.Linear(hidden_size_critic, 1))

    def init_hidden_actor(self):
        return torch.zeros(1, self.n_layers, self.hidden_size_actor)

    def init_hidden_critic(self):
        return torch.zeros(1, self.n_layers, self.hidden_size_critic)

    # ---- the reference forward (dense obs), networks.py:50-69 ----
    def forward(self, observations, actions, hidden_actor=None, hidden_critic=None):
        n, t = observations.shape[:2]
        obs_emb = self.obs_proj(observations.reshape(n, t, -1).float())
        agent_ids = torch.arange(n, device=obs_emb.device)
        return self.forward_emb(obs_emb, actions, hidden_actor, hidden_critic, agent_ids=agent_ids)

    # ---- packed obs -> obs_proj output ----
    def project_packed(self, idx, val):
        """obs_proj(obs.float()) from packed rows: idx u16 / val f32 [..., cap] -> [..., obs_emb_size]."""
        lead = idx.shape[:-1]
        cap = idx.shape[-1]
        out = _PackedProj.apply(idx.reshape(-1, cap).long(), val.reshape(-1, cap), self.obs_proj.weight.t())
        return (out + self.obs_proj.bias).reshape(*lead, -1)

    def forward_emb(self, obs_emb, actions, hidden_actor, hidden_critic, agent_ids=None, starts=None):
        """obs_emb [N, T, E] (obs_proj output), actions [N, T] (last action, -1 = none), hidden [N, 1, H].
        starts [N, T] bool: the recurrent state restarts from zero at these entries (episode starts)."""
        n, t = obs_emb.shape[:2]
        # learner windows with grad: the same layers with their weight gradients as split-K GEMMs (_tall_tn)
        sk = t > 1 and torch.is_grad_enabled()
        mixed = self.mixed(obs_emb, actions, agent_ids, sk)
        ha = hidden_actor[:, 0]
        hc = hidden_critic[:, 0]
        if t == 1 and (starts is None or not bool(starts.any())):  # acting: one fused cell per GRU
            out_p = torch.gru_cell(mixed[:, 0], ha, self.gru_actor.weight_ih_l0, self.gru_actor.weight_hh_l0,
                                   self.gru_actor.bias_ih_l0, self.gru_actor.bias_hh_l0)[:, None]
            out_c = torch.gru_cell(mixed[:, 0], hc, self.gru_critic.weight_ih_l0, self.gru_critic.weight_hh_l0,
                                   self.gru_critic.bias_ih_l0, self.gru_critic.bias_hh_l0)[:, None]
        elif self.gru_window == 'fused':  # a window: both GRUs in one autograd node, GEMMs batched over the window
            keep = torch.ones((n, t), dtype=mixed.dtype, device=mixed.device) if starts is None else \
                (~starts).to(mixed.dtype)
            ga, gc = self.gru_actor, self.gru_critic
            out_p, out_c = _GRUWindow.apply(mixed, keep, ha.detach(), hc.detach(), ga.weight_ih_l0, ga.weight_hh_l0,
                                            ga.bias_ih_l0, ga.bias_hh_l0, gc.weight_ih_l0, gc.weight_hh_l0,
                                            gc.bias_ih_l0, gc.bias_hh_l0)
        elif self.gru_window == 'segments':  # a window: one library RNN call per GRU over the episode segments
            seg = _Segments(starts, n, t, mixed.device)
            out_p = seg.run(self.gru_actor, mixed, ha)
            out_c = seg.run(self.gru_critic, mixed, hc)
        else:  # a window: input gates of all steps as one GEMM, then the fused cell step by step
            keep = None if starts is None else (~starts).to(mixed.dtype)  # [N, T]
            ps, cs = [], []
            for s in range(t):
                if keep is not None:
                    ha = ha * keep[:, s:s + 1]
                    hc = hc * keep[:, s:s + 1]
                ha = torch.gru_cell(mixed[:, s], ha, self.gru_actor.weight_ih_l0, self.gru_actor.weight_hh_l0,
                                    self.gru_actor.bias_ih_l0, self.gru_actor.bias_hh_l0)
                hc = torch.gru_cell(mixed[:, s], hc, self.gru_critic.weight_ih_l0, self.gru_critic.weight_hh_l0,
                                    self.gru_critic.bias_ih_l0, self.gru_critic.bias_hh_l0)
                ps.append(ha)
                cs.append(hc)
            out_p, out_c = torch.stack(ps, 1), torch.stack(cs, 1)
        return self._heads(out_p, out_c, sk)

    def mixed(self, obs_emb, actions, agent_ids=None, sk=False):
        """The GRUs' input: mix(cat(obs_emb, [agent_emb,] action_emb)) (networks.py:52-58); sk = the learner's
        split-K weight gradients."""
        n, t = obs_emb.shape[:2]
        action_emb = _Embed.apply(actions + 1, self.action_emb.weight, self.action_emb.padding_idx) if sk else \
            self.action_emb(actions + 1)  # shift by one: padding idx (networks.py:53)
        if not self.use_agent_embedding:
            x_t = torch.cat((obs_emb, action_emb), -1)
        else:
            ids = agent_ids if agent_ids is not None else torch.arange(n, device=obs_emb.device)
            agent_emb = self.agent_emb(ids.view(-1, 1).expand(n, t))
            x_t = torch.cat((obs_emb, agent_emb, action_emb), -1)
        if sk:
            return _lin(self.mix[3], torch.tanh(_lin(self.mix[1], torch.tanh(x_t))))
        return self.mix(x_t)

    def _heads(self, out_p, out_c, sk):
        if sk:
            logits = _lin(self.action_head[2], torch.tanh(_lin(self.action_head[0], out_p)))
            critic = _lin(self.critic_head[2], torch.tanh(_lin(self.critic_head[0], out_c))).squeeze(-1)
        else:
            logits = self.action_head(out_p)
            critic = self.critic_head(out_c).squeeze(-1)
        return dict(logits=logits, critic=critic, hidden_actor=out_p, hidden_critic=out_c)


class _Segments:
    """The episode segments of a window: row r restarts its recurrent state from zero at every entry s with
    starts[r, s] (an episode start inside the window, base_ac.py:98-100 resets at env.reset()). Every segment
    becomes one sequence of a packed batch (its initial state: the row's carried state, or zero after a
    restart), so nn.GRU runs the whole window in one library call (MIOpen) instead of T cell steps, and the
    outputs are scattered back to [N, T, H]. One host synchronisation (the segment count) per window."""

    def __init__(self, starts, n, t, device):
        st = torch.zeros((n, t), dtype=torch.bool, device=device) if starts is None else starts.clone()
        st[:, 0] = True
        pos = st.nonzero()  # [S, 2] (row, start), rows ascending, starts ascending within a row
        self.rows, a = pos[:, 0], pos[:, 1]
        s_n = pos.shape[0]
        nxt = torch.full((s_n,), t, dtype=torch.long, device=device)
        if s_n > 1:
            same = self.rows[1:] == self.rows[:-1]
            nxt[:-1] = torch.where(same, a[1:], torch.full_like(a[1:], t))
        self.len = nxt - a  # >= 1
        k = torch.arange(t, device=device)
        self.valid = k[None, :] < self.len[:, None]  # [S, T]
        self.src = (self.rows[:, None] * t + (a[:, None] + k[None, :]).clamp(max=t - 1))  # flat (row, time)
        # the carried state only for a row's first segment, unless the row restarts at entry 0 too
        self.first = (a == 0) if starts is None else (a == 0) & ~starts[self.rows, 0]
        self.n, self.t = n, t
        self.len_cpu = self.len.cpu()

    def run(self, gru, x, h0):
        from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence
        n, t = self.n, self.t
        xf = x.reshape(n * t, -1)
        xs = xf[self.src] * self.valid[..., None].to(x.dtype)  # [S, T, I]
        hs = torch.where(self.first[:, None], h0[self.rows], torch.zeros_like(h0[self.rows]))
        packed = pack_padded_sequence(xs, self.len_cpu, batch_first=True, enforce_sorted=False)
        out, _ = gru(packed, hs[None].contiguous())
        out, _ = pad_packed_sequence(out, batch_first=True, total_length=t)  # [S, T, H]
        dst = self.src[self.valid]
        res = torch.zeros((n * t, out.shape[-1]), dtype=out.dtype, device=out.device)
        res = res.index_copy(0, dst, out[self.valid])
        return res.view(n, t, -1)


class _PackedProj(torch.autograd.Function):
    """x @ W^T over packed rows: forward is a gather-sum of W^T rows (embedding_bag); the weight gradient is
    D^T @ G with D the rows scattered back to dense, one GEMM (embedding_bag's own backward scatters
    M x cap x E atomics onto the K x E table, ~100x slower at M = 393K rows)."""

    @staticmethod
    def forward(ctx, idx, val, wt):
        ctx.save_for_backward(idx, val)
        ctx.k = wt.shape[0]
        return F.embedding_bag(idx, wt, per_sample_weights=val, mode='sum')

    @staticmethod
    def backward(ctx, g):
        idx, val = ctx.saved_tensors
        return None, None, _packed_weight_grad(idx, val, g, ctx.k)


def _packed_weight_grad(idx, val, g, k):
    """D^T @ g for the packed rows (idx, val) [M, cap] scattered to dense D [M, k]: one GEMM per block of rows
    (<= 512 MiB of dense rows), instead of embedding_bag's M x cap x E atomics onto the k x E table."""
    gw = torch.zeros((k, g.shape[1]), dtype=g.dtype, device=g.device)
    step = max(1, (1 << 27) // max(k, 1))
    for r0 in range(0, idx.shape[0], step):
        d = torch.zeros((min(step, idx.shape[0] - r0), k), dtype=g.dtype, device=g.device)
        d.scatter_add_(1, idx[r0:r0 + step], val[r0:r0 + step].to(g.dtype))
        gw += _tall_tn(d, g[r0:r0 + step])
    return gw


def _project_dense(idx, val, proj):
    """obs_proj over packed rows without grad: the rows scattered to dense blocks (<= 512 MiB) and one GEMM each
    (embedding_bag with per-sample weights ran 0.77 ms for C3's 65,536 rows on the MI355X)."""
    lead, cap = idx.shape[:-1], idx.shape[-1]
    idx2, val2 = idx.reshape(-1, cap).long(), val.reshape(-1, cap)
    k = proj.weight.shape[1]
    out = torch.empty((idx2.shape[0], proj.weight.shape[0]), dtype=proj.weight.dtype, device=idx2.device)
    step = max(1, (1 << 27) // max(k, 1))
    for r0 in range(0, idx2.shape[0], step):
        d = torch.zeros((min(step, idx2.shape[0] - r0), k), dtype=proj.weight.dtype, device=idx2.device)
        d.scatter_add_(1, idx2[r0:r0 + step], val2[r0:r0 + step].to(d.dtype))
        torch.addmm(proj.bias, d, proj.weight.t(), out=out[r0:r0 + step])
    return out.view(*lead, -1)


class _EngineProj(torch.autograd.Function):
    """obs_proj(obs) for the learner, forward taken from the engine: every slot of the window was rendered with
    the current weights (the fused projection of k_obs, MFG_OBS_PACKED), so the forward is that output (bias
    included) and only the backward touches the packed rows (weight: D^T g, bias: the row sum of g)."""

    @staticmethod
    def forward(ctx, idx, val, weight, bias, emb):
        ctx.save_for_backward(idx, val)
        ctx.k = weight.shape[1]
        return emb.clone()

    @staticmethod
    def backward(ctx, g):
        idx, val = ctx.saved_tensors
        gw, gb = _packed_grads(idx, val, g, ctx.k)
        return None, None, gw, gb, None


def _packed_grads(idx, val, g, k):
    """obs_proj's (weight [E, k], bias [E]) gradients from packed rows idx / val [M, cap] and g [M, E]: D^T g with D
    the rows made dense (on the GPU by mfg_packed_densify, include/mfg_learn.h: one coalesced pass, no zero fill
    or scatter_add), one split-K GEMM per block of <= 512 MiB of dense rows, and the column sums of g."""
    if not (g.is_cuda and idx.dtype == torch.uint16) or k > _DENSIFY_MAX_K:
        # (k past the densify kernel's wave-private LDS row: the same dense rows by scatter_add on the device)
        return _packed_weight_grad(idx.long(), val, g, k).t(), g.sum(0)
    L, st = _gru_lib(), torch.cuda.current_stream(g.device).cuda_stream
    idx, val = idx.contiguous(), val.contiguous()
    gw = None
    step = max(1, (1 << 27) // max(k, 1))
    for r0 in range(0, idx.shape[0], step):
        rows = min(step, idx.shape[0] - r0)
        d = torch.empty((rows, k), dtype=g.dtype, device=g.device)
        if L.mfg_packed_densify(idx[r0].data_ptr(), val[r0].data_ptr(), rows, idx.shape[1], k, d.data_ptr(), k, st):
            raise RuntimeError('mfg_packed_densify failed')
        part = _tall_tn(g[r0:r0 + rows], d)  # [E, k]
        gw = part if gw is None else gw + part
    return gw, g.sum(0)


_GRU_LIB = None
_DENSIFY_MAX_K = 4096  # mfg_packed_densify's bound on the dense row length (include/mfg_learn.h)


def _gru_lib():
    """libmfg_hip.so's learner kernels (include/mfg_learn.h), bound once."""
    global _GRU_LIB
    if _GRU_LIB is None:
        import ctypes as C
        from .engine import load_lib
        L = load_lib()
        p, i64 = C.c_void_p, C.c_int64
        L.mfg_gru_fwd_step.argtypes = [p, i64, p, p, p, i64, p, i64, p, i64, p, p, p, p, p, i64, i64, C.c_int, p]
        L.mfg_gru_fwd_step.restype = C.c_int
        L.mfg_gru_bwd_step.argtypes = [p, i64, p, p, i64, p, p, p, p, p, i64, p, i64, p, i64, p, i64, C.c_int, p]
        L.mfg_gru_bwd_step.restype = C.c_int
        L.mfg_packed_densify.argtypes = [p, p, i64, C.c_int, C.c_int, p, i64, p]
        L.mfg_packed_densify.restype = C.c_int
        L.mfg_packed_project.argtypes = [p, p, i64, C.c_int, p, p, C.c_int, C.c_int, p, i64, p]
        L.mfg_packed_project.restype = C.c_int
        L.mfg_sample_categorical.argtypes = [p, i64, C.c_int, p, i64, p, p]
        L.mfg_sample_categorical.restype = C.c_int
        _GRU_LIB = L
    return _GRU_LIB


def _use_gru_kernels(x):
    """The learner's GRU window runs its elementwise steps as HIP kernels on the GPU (fp32); CPU tensors take the
    tensor code (the same formulas)."""
    return x.is_cuda and x.dtype == torch.float32


def _ptr(t):
    return None if t is None else t.data_ptr()


class _GRUWindow(torch.autograd.Function):
    """Both GRUs of RecurrentAC (layer 0, PyTorch gate order r, z, n) over a window of T steps with per-entry
    restarts, forward and backward written out so the GEMMs are batched over the window:
      forward:  the input gates of every step and both GRUs as ONE GEMM [N*T, I] x [I, 3Ha + 3Hc]; per step the
                recurrent gates h W_hh^T (one GEMM per GRU, the only sequential part);
      backward: per step the recurrent chain dh W_hh (one GEMM per GRU), then ONE GEMM each for the input-weight
                gradient of both GRUs, the input gradient, and per GRU one recurrent-weight gradient over all N*T
                rows (autograd over T fused cells issues 4 GEMMs per step and GRU: 48 instead of 10 at T = 6).
    keep [N, T]: the state entering step s is h_{s-1} * keep[:, s] (0 = an episode restart at s). h0 gets no
    gradient (the learner's carried state is detached, base_ac.py:126-128)."""

    @staticmethod
    def forward(ctx, x, keep, h0a, h0c, wia, wha, bia, bha, wic, whc, bic, bhc):
        n, t, i_dim = x.shape
        ha_dim, hc_dim = wha.shape[1], whc.shape[1]
        wi = torch.cat([wia, wic], 0)  # [3Ha + 3Hc, I]
        bi = torch.cat([bia, bic], 0)
        gi = torch.addmm(bi, x.reshape(n * t, i_dim), wi.t()).view(n, t, -1)
        outs, saved = [], []
        if _use_gru_kernels(x):  # per step: the recurrent GEMM + one fused elementwise kernel (mfg_gru_fwd_step)
            L, st = _gru_lib(), torch.cuda.current_stream(x.device).cuda_stream
            keep = keep.contiguous()
            g_all = gi.shape[-1]
            for (h, wh, bh, lo, hd) in ((h0a, wha, bha, 0, ha_dim), (h0c, whc, bhc, 3 * ha_dim, hc_dim)):
                hs = torch.empty((n, t, hd), dtype=x.dtype, device=x.device)
                sv = torch.empty((5, n, t, hd), dtype=x.dtype, device=x.device)  # hp, r, z, n, gh_n
                bh = bh.contiguous()
                hcur, h_row = h.contiguous(), hd
                for s in range(t):
                    gh0 = hcur @ wh.t()
                    rc = L.mfg_gru_fwd_step(gi[:, s, lo:].data_ptr(), t * g_all, gh0.data_ptr(), bh.data_ptr(),
                                            hcur.data_ptr(), h_row, keep[:, s].data_ptr(), t, hs[:, s].data_ptr(),
                                            t * hd, sv[0, :, s].data_ptr(), sv[1, :, s].data_ptr(),
                                            sv[2, :, s].data_ptr(), sv[3, :, s].data_ptr(), sv[4, :, s].data_ptr(),
                                            t * hd, n, hd, st)
                    if rc:
                        raise RuntimeError('mfg_gru_fwd_step failed')
                    hcur, h_row = hs[:, s], t * hd
                outs.append(hs)
                saved += list(sv.unbind(0))
            ctx.save_for_backward(x, keep, wi, wha, whc, *saved)
            ctx.dims = (ha_dim, hc_dim)
            return outs[0], outs[1]
        for (h, wh, bh, lo, hd) in ((h0a, wha, bha, 0, ha_dim), (h0c, whc, bhc, 3 * ha_dim, hc_dim)):
            hs, hps, rs, zs, ns, ghns = [], [], [], [], [], []
            for s in range(t):
                hp = h * keep[:, s:s + 1]
                gh = torch.addmm(bh, hp, wh.t())
                g = gi[:, s, lo:lo + 3 * hd]
                r = torch.sigmoid(g[:, :hd] + gh[:, :hd])
                z = torch.sigmoid(g[:, hd:2 * hd] + gh[:, hd:2 * hd])
                ghn = gh[:, 2 * hd:]
                nn_ = torch.tanh(g[:, 2 * hd:] + r * ghn)
                h = nn_ + z * (hp - nn_)  # (1 - z) n + z h
                hs.append(h); hps.append(hp); rs.append(r); zs.append(z); ns.append(nn_); ghns.append(ghn)
            outs.append(torch.stack(hs, 1))
            saved += [torch.stack(v, 1) for v in (hps, rs, zs, ns, ghns)]
        ctx.save_for_backward(x, keep, wi, wha, whc, *saved)
        ctx.dims = (ha_dim, hc_dim)
        return outs[0], outs[1]

    @staticmethod
    def backward(ctx, douta, doutc):
        x, keep, wi, wha, whc, *saved = ctx.saved_tensors
        ha_dim, hc_dim = ctx.dims
        n, t, i_dim = x.shape
        dgis, grads = [], []
        gpu = _use_gru_kernels(x)
        g_all = 3 * (ha_dim + hc_dim)
        # GPU: both GRUs' input-gate gradients straight into one [n, t, 3Ha + 3Hc] buffer (no concatenation)
        dgi_all = torch.empty((n, t, g_all), dtype=x.dtype, device=x.device) if gpu else None
        for gi_idx, (dout, wh, hd) in enumerate(((douta, wha, ha_dim), (doutc, whc, hc_dim))):
            hps, rs, zs, ns, ghns = saved[5 * gi_idx:5 * gi_idx + 5]
            if gpu:  # per step: one fused elementwise kernel (mfg_gru_bwd_step) + the recurrent GEMM
                L, st = _gru_lib(), torch.cuda.current_stream(x.device).cuda_stream
                dgi = dgi_all[:, :, 3 * ha_dim * gi_idx:]
                dgh = torch.empty((n, t, 3 * hd), dtype=x.dtype, device=x.device)
                dout = None if dout is None else dout.contiguous()
                sv_row = hps.stride(0)
                dhp = None
                for s in range(t - 1, -1, -1):
                    dhz = torch.empty((n, hd), dtype=x.dtype, device=x.device)
                    rc = L.mfg_gru_bwd_step(None if dout is None else dout[:, s].data_ptr(), t * hd, _ptr(dhp),
                                            None if dhp is None else keep[:, s + 1].data_ptr(), t,
                                            rs[:, s].data_ptr(), zs[:, s].data_ptr(), ns[:, s].data_ptr(),
                                            ghns[:, s].data_ptr(), hps[:, s].data_ptr(), sv_row,
                                            dgi[:, s].data_ptr(), t * g_all, dgh[:, s].data_ptr(), t * 3 * hd,
                                            dhz.data_ptr(), n, hd, st)
                    if rc:
                        raise RuntimeError('mfg_gru_bwd_step failed')
                    dhp = torch.addmm(dhz, dgh[:, s], wh)
                dgh2 = dgh.reshape(n * t, 3 * hd)
                grads.append((_tall_tn(dgh2, hps.reshape(n * t, hd)), dgh2.sum(0)))
                continue
            dgi = torch.empty((n, t, 3 * hd), dtype=x.dtype, device=x.device)
            dgh = torch.empty_like(dgi)
            carry = torch.zeros((n, hd), dtype=x.dtype, device=x.device)
            for s in range(t - 1, -1, -1):
                dh = carry if dout is None else dout[:, s] + carry
                r, z, nn_, ghn, hp = rs[:, s], zs[:, s], ns[:, s], ghns[:, s], hps[:, s]
                dn = dh * (1.0 - z) * (1.0 - nn_ * nn_)
                dz = dh * (hp - nn_) * z * (1.0 - z)
                dr = dn * ghn * r * (1.0 - r)
                dgi[:, s, :hd] = dr
                dgi[:, s, hd:2 * hd] = dz
                dgi[:, s, 2 * hd:] = dn
                dgh[:, s, :hd] = dr
                dgh[:, s, hd:2 * hd] = dz
                dgh[:, s, 2 * hd:] = dn * r
                dhp = torch.addmm(dh * z, dgh[:, s], wh)  # dh z + dgh W_hh
                carry = dhp * keep[:, s:s + 1]
            dgis.append(dgi)
            dgh2 = dgh.reshape(n * t, 3 * hd)
            grads.append((_tall_tn(dgh2, hps.reshape(n * t, hd)), dgh2.sum(0)))  # dW_hh, db_hh
        dgi_all = (dgi_all if gpu else torch.cat(dgis, 2)).reshape(n * t, -1)
        dwi = _tall_tn(dgi_all, x.reshape(n * t, i_dim))  # [3Ha + 3Hc, I]
        dbi = dgi_all.sum(0)
        dx = (dgi_all @ wi).view(n, t, i_dim)
        sa = 3 * ha_dim
        return (dx, None, None, None, dwi[:sa], grads[0][0], dbi[:sa], grads[0][1],
                dwi[sa:], grads[1][0], dbi[sa:], grads[1][1])


class _MixSaved(torch.autograd.Function):
    """RecurrentAC.mix (Tanh, Linear, Tanh, Linear; networks.py:24-25) over a window whose forward the acting steps
    already ran with the same weights: saved = (ax, h1, mixed, a_prev, pad), ax = tanh(cat(obs_emb, action_emb))
    [M, E + AE], h1 = tanh(ax W1^T + b1) [M, H], mixed [M, H] and the action inputs a_prev [M] (-1 = none). The
    forward returns the stored output; the backward is the layers' chain rule (weight gradients by _tall_tn), with
    the obs_emb gradient for obs_proj and the action-embedding gradient as onehot(a_prev + 1)^T g (padding row 0)."""

    @staticmethod
    def forward(ctx, emb, w1, b1, w3, b3, aw, saved):
        ax, h1, mx, a_prev, pad = saved
        ctx.save_for_backward(w1, w3, ax, h1, a_prev)
        ctx.e_dim, ctx.n_emb, ctx.pad = emb.shape[1], aw.shape[0], pad
        return mx.view_as(mx)

    @staticmethod
    def backward(ctx, g3):
        w1, w3, ax, h1, a_prev = ctx.saved_tensors
        g3 = g3.contiguous()
        dw3, db3 = _tall_tn(g3, h1), g3.sum(0)
        dz1 = torch.ops.aten.tanh_backward(g3 @ w3, h1)  # g (1 - h1^2), one kernel
        dw1, db1 = _tall_tn(dz1, ax), dz1.sum(0)
        dx = torch.ops.aten.tanh_backward(dz1 @ w1, ax)
        e = ctx.e_dim
        oh = F.one_hot(a_prev + 1, ctx.n_emb).to(dx.dtype)
        daw = _tall_tn(oh, dx[:, e:].contiguous())
        if ctx.pad is not None:
            daw[ctx.pad] = 0
        return dx[:, :e], dw1, db1, dw3, db3, daw, None


class _GRUWindowSavedT(torch.autograd.Function):
    """Both GRUs over a window whose forward the acting steps already ran (mfg_gru_fwd_step) with the same weights,
    entry-major: saved = (hs_a, hs_c, sv_a, sv_c), outputs [T, N, H] and gate activations [5, T, N, H] (hp, r, z, n,
    gh_n); x [T*N, I] the GRUs' input, keep [T, N] (0 = an episode restart at that entry). The forward returns the
    stored outputs; the backward is _GRUWindow's (per step one mfg_gru_bwd_step and the recurrent GEMM, then one GEMM
    each for the input-weight, input and recurrent-weight gradients over all T*N rows) on entry-major rows."""

    @staticmethod
    def forward(ctx, x, keep, saved, wia, wha, bia, bha, wic, whc, bic, bhc):
        hs_a, hs_c, sv_a, sv_c = saved
        wi = torch.cat([wia, wic], 0)
        ctx.save_for_backward(x, keep, wi, wha, whc, *sv_a.unbind(0), *sv_c.unbind(0))
        t, n = keep.shape
        return hs_a.view(t * n, -1), hs_c.view(t * n, -1)

    @staticmethod
    def backward(ctx, douta, doutc):
        x, keep, wi, wha, whc, *sv = ctx.saved_tensors
        t, n = keep.shape
        ha_dim, hc_dim = wha.shape[1], whc.shape[1]
        g_all = 3 * (ha_dim + hc_dim)
        L, st = _gru_lib(), torch.cuda.current_stream(x.device).cuda_stream
        dgi_all = torch.empty((t, n, g_all), dtype=x.dtype, device=x.device)
        grads = []
        for gidx, (dout, wh, hd) in enumerate(((douta, wha, ha_dim), (doutc, whc, hc_dim))):
            hps, rs, zs, ns, ghns = sv[5 * gidx:5 * gidx + 5]
            dgh = torch.empty((t, n, 3 * hd), dtype=x.dtype, device=x.device)
            dout = None if dout is None else dout.contiguous().view(t, n, hd)
            lo = 3 * ha_dim * gidx
            dhp = None
            for s in range(t - 1, -1, -1):
                dhz = torch.empty((n, hd), dtype=x.dtype, device=x.device)
                rc = L.mfg_gru_bwd_step(None if dout is None else dout[s].data_ptr(), hd, _ptr(dhp),
                                        None if dhp is None else keep[s + 1].data_ptr(), 1,
                                        rs[s].data_ptr(), zs[s].data_ptr(), ns[s].data_ptr(), ghns[s].data_ptr(),
                                        hps[s].data_ptr(), hd, dgi_all[s, :, lo:].data_ptr(), g_all,
                                        dgh[s].data_ptr(), 3 * hd, dhz.data_ptr(), n, hd, st)
                if rc:
                    raise RuntimeError('mfg_gru_bwd_step failed')
                dhp = torch.addmm(dhz, dgh[s], wh)
            dgh2 = dgh.view(t * n, 3 * hd)
            grads.append((_tall_tn(dgh2, hps.reshape(t * n, hd)), dgh2.sum(0)))
        dgi2 = dgi_all.view(t * n, g_all)
        dwi, dbi = _tall_tn(dgi2, x), dgi2.sum(0)
        dx = dgi2 @ wi
        sa = 3 * ha_dim
        return (dx, None, None, dwi[:sa], grads[0][0], dbi[:sa], grads[0][1], dwi[sa:], grads[1][0], dbi[sa:],
                grads[1][1])


def _gru_cell(gi, h, gru):
    """One nn.GRU step (layer 0) from precomputed input gates gi = x W_ih^T + b_ih."""
    gh = F.linear(h, gru.weight_hh_l0, gru.bias_hh_l0)
    i_r, i_z, i_n = gi.chunk(3, -1)
    h_r, h_z, h_n = gh.chunk(3, -1)
    r = torch.sigmoid(i_r + h_r)
    z = torch.sigmoid(i_z + h_z)
    n = torch.tanh(i_n + r * h_n)
    return (1.0 - z) * n + z * h


def compute_advantages(critic, reward, done, gamma, gae_coef=0.0):
    """base_ac.py:185-198."""
    tds = (reward + gamma * (1.0 - done) * critic[:, 1:].detach()) - critic[:, :-1]
    if gae_coef <= 0:
        return tds
    gae = torch.zeros_like(tds[:, -1])
    gaes = []
    for t in range(tds.shape[1] - 1, -1, -1):
        gae = tds[:, t] + gamma * gae_coef * (1.0 - done[:, t]) * gae
        gaes.insert(0, gae)
    return torch.stack(gaes, dim=1)


def a2c_loss(out, actions, reward, done, gamma, entropy_coef, vf_coef, gae_coef=0.0):
    """base_ac.py:200-217 on a forward output: actions [N, T+1] (entry 0 = the action before the window),
    reward / done [N, T] (the targets of entries 1..T)."""
    return a2c_loss_terms(out['logits'][:, :-1], out['critic'], actions, reward, done, gamma, entropy_coef, vf_coef,
                          gae_coef)


def a2c_loss_terms(logits, critic, actions, reward, done, gamma, entropy_coef, vf_coef, gae_coef=0.0):
    """a2c_loss on the policy logits of entries 0..T-1 [N, T, n_act] and the critic of entries 0..T [N, T+1]."""
    entropy_loss = Categorical(logits=logits, validate_args=False).entropy().mean(-1)
    advantages = compute_advantages(critic, reward, done, gamma, gae_coef)
    value_loss = advantages.pow(2).mean(-1)
    log_ap = torch.log_softmax(logits, -1)
    log_ap = torch.gather(log_ap, dim=-1, index=actions[:, 1:].unsqueeze(-1)).squeeze(-1)
    a2c = -(advantages.detach() * log_ap).mean(-1)
    loss = a2c + vf_coef * value_loss - entropy_coef * entropy_loss
    return loss.mean()


class BatchedA2C:
    """A2C with a shared ``RecurrentAC`` over B envs x A agents of one engine, everything on the device.

    Per step: the engine renders o_t as packed rows + the fused ``obs_proj`` (one kernel, no dense obs); the
    policy acts on (o_t, a_{t-1}, h_t); actions go straight back into ``mfg_step`` (int32 on the device).
    Every ``n_steps`` steps: one A2C update on the window o_0..o_T (``base_ac.py:126-128``). obs_proj's forward is
    the render's own fused output (every slot was rendered with the current weights; ``engine_emb=False``
    re-evaluates it by ``embedding_bag`` over the stored entries), its backward runs on the stored entries. No host
    synchronisation inside ``step``;
    ``learn`` syncs once when ``check_cap`` is set (truncated packed rows raise).

    ``reuse_acting=True`` (the default on the GPU, without the agent embedding): the weights are fixed over a window, so
    the acting steps' forward is the learner's forward of entries 0..T-1. Acting runs the mix and both GRUs itself
    (``mfg_gru_fwd_step``) and keeps every activation in entry-major window buffers; the learner evaluates the heads
    and the loss with grad and runs the mix / GRU backward on the stored activations (``_MixSaved``,
    ``_GRUWindowSavedT``), plus one no-grad critic step for the bootstrap entry T. ``_loss_recompute`` is the
    reference learner's full-window recompute (pinned equal). Sampling on the GPU is ``mfg_sample_categorical`` (a
    row with non-finite logits is marked -1 and ``learn`` raises when ``check_cap`` is set).

    ``graph=True``: the update (loss, backward, gradient clipping, RMSprop step and the window slide, ~1,300 launches)
    is captured once as a HIP graph after two eager warm-up updates on a side stream and replayed from then on (one
    launch per update); the optimizer then keeps its step counters on the device (``capturable``).

    Read at window boundaries: ``episodes`` and ``reward_sum`` fold in a window's done flags and rewards in ``learn``
    (once per window), so a monitor that reads them between two ``learn`` calls sees the previous window's totals.
    The engine's floor-shuffle replay is deferred to the window's last step (``MFG_STEP_DEFER_REPLAY``): a state
    snapshot (``export_state``) taken mid-window holds a non-reference MT state and floor order until that replay
    (the step results are identical either way)."""

    def __init__(self, factory, net=None, n_steps=5, gamma=0.99, entropy_coef=0.01, vf_coef=0.5, gae_coef=0.0,
                 lr=3e-4, cap=32, obs_emb_size=96, action_emb_size=16, hidden_size=64, use_agent_embedding=False,
                 check_cap=True, generator=None, engine_emb=True, graph=False, act_graph=False, reuse_acting=True):
        from .engine import PackedObs
        self.f = factory
        eng = factory.engine
        spec = factory.spec
        self.B, self.A = eng.B, eng.A
        self.N = self.B * self.A
        self.dev = eng.device
        n_act = set(int(x) for x in spec.n_actions)
        if len(n_act) != 1:
            raise ValueError('BatchedA2C shares one network: all agents need the same number of actions')
        self.n_actions = n_act.pop()
        kdim = eng.lmax * eng.obs_hw[0] * eng.obs_hw[1]
        if not check_cap and cap < kdim:
            # a truncated row would make acting (the fused emb sums every nonzero entry) and learning (the stored
            # cap entries only) see different obs_proj inputs: skipping the check is allowed only when no row
            # can be truncated
            raise ValueError(f'check_cap=False needs cap >= lmax*h*w = {kdim} (rows can hold up to that many '
                             f'nonzero entries); got cap {cap}')
        self.net = net if net is not None else RecurrentAC(
            kdim, self.n_actions, obs_emb_size, action_emb_size, hidden_size, hidden_size, self.A,
            use_agent_embedding=use_agent_embedding)
        self.net.to(self.dev)
        self.graph = bool(graph)
        # act_graph: each window slot's policy step (forward, sampling, action copy) captured as a HIP graph after two
        # eager warm-ups (not with an explicit generator: its draws stay on the eager path)
        self.act_graph = bool(act_graph) and generator is None
        self._act_graphs, self._act_warm = {}, {}
        self.opt = torch.optim.RMSprop(self.net.parameters(), lr=lr, eps=1e-5, capturable=self.graph)
        self._graph, self._warm = None, 0
        self.T, self.gamma, self.entropy_coef, self.vf_coef, self.gae_coef = n_steps, gamma, entropy_coef, \
            vf_coef, gae_coef
        self.check_cap = check_cap
        self.engine_emb = engine_emb  # learner forward of obs_proj: the engine's fused output (True) or a gather
        self.gen = generator
        T, N, dev = self.T, self.N, self.dev
        # obs slots o_0..o_T of the window (entries + fused projection), written by the engine
        self.pobs = PackedObs(eng, K=T + 1, cap=cap, weight=self.net.obs_proj.weight, bias=self.net.obs_proj.bias)
        self.slot = [self.pobs.view(k) for k in range(T + 1)]
        self.act_in = torch.full((T + 1, self.B, self.A), -1, dtype=torch.int64, device=dev)  # a_{t-1}, -1 = none
        self.act = torch.zeros((T, self.B, self.A), dtype=torch.int32, device=dev)
        self.rew = torch.zeros((T, self.B, self.A), dtype=torch.float64, device=dev)
        self.done = torch.zeros((T, self.B), dtype=torch.uint8, device=dev)
        H = self.net.hidden_size_actor
        self.h0a = torch.zeros((N, 1, H), device=dev)  # hidden state fed at entry 0 of the window
        self.h0c = torch.zeros((N, 1, self.net.hidden_size_critic), device=dev)
        self.ha, self.hc = self.h0a.clone(), self.h0c.clone()  # persistent: updated in place (graph inputs)
        self._ha_new, self._hc_new = self.h0a.clone(), self.h0c.clone()  # the policy step's new states (static)
        # reuse_acting: the acting steps run both GRUs through mfg_gru_fwd_step and keep every entry's outputs and
        # gate activations (the weights are fixed over a window, so they ARE the learner's recurrent forward of
        # entries 0..T-1); the learner then evaluates only the input layers, heads and loss with grad, the entry-T
        # bootstrap critic without grad, and runs the GRU backward on the stored activations (no window recompute)
        # (entry-major [T, N, ...] window buffers: an acting step writes one contiguous slice, and the learner's rows
        # are the engine's slot order, so the packed rows and fused projection of the window are used in place)
        self.reuse = bool(reuse_acting) and self.dev.type == 'cuda' and not self.net.use_agent_embedding
        if self.reuse:
            Ha, Hc = H, self.net.hidden_size_critic
            E, AE = self.net.obs_proj.weight.shape[0], self.net.action_emb_size
            Hm = self.net.mix[1].weight.shape[0]
            self.ax = torch.zeros((T, N, E + AE), device=dev)  # tanh(cat(obs_emb, action_emb)), the mix input
            self.h1 = torch.zeros((T, N, Hm), device=dev)  # the mix's hidden tanh
            self.mx = torch.zeros((T, N, self.net.mix[3].weight.shape[0]), device=dev)  # the GRUs' input
            self.hs_a = torch.zeros((T, N, Ha), device=dev)
            self.hs_c = torch.zeros((T, N, Hc), device=dev)
            self.sv_a = torch.zeros((5, T, N, Ha), device=dev)  # hp, r, z, n, gh_n
            self.sv_c = torch.zeros((5, T, N, Hc), device=dev)
            self._one = torch.ones(1, device=dev)
        self._u = torch.empty(N, device=dev)  # the sampling uniforms (static: graph-captured acting)
        self.last_loss = torch.zeros((), device=dev)
        self.agent_ids = torch.arange(self.A, device=dev).repeat(self.B)
        self.t = 0
        self.updates = 0
        self.episodes = torch.zeros((), dtype=torch.float64, device=dev)  # finished episodes, counted per window
        self.reward_sum = torch.zeros((), dtype=torch.float64, device=dev)
        self._started = False

    def reset(self):
        self.f.engine.reset(obs=self.slot[0], init=0 if self.f._created else 1, seed_base=self.f.seed_base)
        self.f._created = True
        self._started = True
        self.t = 0

    @torch.no_grad()
    def step(self):
        """One env-step of every env with the current policy (no host sync)."""
        if not self._started:
            self.reset()
        t = self.t
        self._policy_step(t)
        # the shuffle-debt replay once per window, at its last step (MFG_STEP_DEFER_REPLAY)
        self.f.engine.step(1, actions=self.act[t], reward=self.rew[t], done=self.done[t], obs=self.slot[t + 1],
                           auto_reset=True, step_base=self.f.t, defer_replay=t + 1 < self.T)
        self.f.t += 1
        d = self.done[t].bool()
        # the next entry's inputs: last action (-1 after an episode end) and the recurrent state (zero then)
        a = self.act[t].long()
        self.act_in[t + 1].copy_(torch.where(d.view(-1, 1), torch.full_like(a, -1), a))
        keep = (~d).to(self.ha.dtype).view(self.B, 1, 1)  # broadcast over the env's agents
        ha_new, hc_new = (self.hs_a[t], self.hs_c[t]) if self.reuse else (self._ha_new, self._hc_new)
        torch.mul(ha_new.view(self.B, self.A, -1), keep, out=self.ha.view(self.B, self.A, -1))
        torch.mul(hc_new.view(self.B, self.A, -1), keep, out=self.hc.view(self.B, self.A, -1))
        self.t += 1
        if self.t == self.T:
            self.learn()

    @torch.no_grad()
    def _policy(self, t):
        """Acting at window slot t: the policy on (o_t, a_{t-1}, h_t), an action per agent into act[t], the new
        recurrent states into the static _ha_new / _hc_new (reuse_acting: the mix activations into ax / h1 / mx [t],
        the recurrent states into hs_a / hs_c [t] and the gate activations into sv_a / sv_c [:, t]; the critic head
        is the learner's alone then)."""
        emb = self.pobs.emb[t].view(self.N, 1, -1)
        a_in = self.act_in[t].view(self.N, 1)
        if self.reuse:
            net, e = self.net, emb.shape[-1]
            ax, h1, mx = self.ax[t], self.h1[t], self.mx[t]
            # tanh(cat(obs_emb, action_emb)) as two writes into the slot (tanh is elementwise); then the two layers
            torch.tanh(emb[:, 0], out=ax[:, :e])
            ax[:, e:].copy_(torch.tanh(net.action_emb.weight)[self.act_in[t].view(-1) + 1])
            torch.tanh(torch.addmm(net.mix[1].bias, ax, net.mix[1].weight.t()), out=h1)
            torch.addmm(net.mix[3].bias, h1, net.mix[3].weight.t(), out=mx)
            self._gru_step(mx, t)
            self._sample(net.action_head(self.hs_a[t]), t)
            return
        out = self.net.forward_emb(emb, a_in, self.ha, self.hc, agent_ids=self.agent_ids)
        self._sample(out['logits'][:, 0], t)
        self._ha_new.copy_(out['hidden_actor'])
        self._hc_new.copy_(out['hidden_critic'])

    def _gru_step(self, x, t):
        """Both GRU cells of entry t on x [N, I] (one input-gate GEMM for both, one recurrent GEMM and one
        mfg_gru_fwd_step each), storing outputs and activations at entry t of the window buffers."""
        net, N, T = self.net, self.N, self.T
        ga, gc = net.gru_actor, net.gru_critic
        gi = torch.addmm(torch.cat([ga.bias_ih_l0, gc.bias_ih_l0]), x, torch.cat([ga.weight_ih_l0, gc.weight_ih_l0]).t())
        L, st = _gru_lib(), torch.cuda.current_stream(self.dev).cuda_stream
        lo = 0
        for (h, gru, hs, sv) in ((self.ha, ga, self.hs_a, self.sv_a), (self.hc, gc, self.hs_c, self.sv_c)):
            hd = hs.shape[-1]
            h2 = h[:, 0]
            gh0 = h2 @ gru.weight_hh_l0.t()
            rc = L.mfg_gru_fwd_step(gi[:, lo:].data_ptr(), gi.shape[1], gh0.data_ptr(), gru.bias_hh_l0.data_ptr(),
                                    h2.data_ptr(), hd, self._one.data_ptr(), 0, hs[t].data_ptr(), hd,
                                    sv[0, t].data_ptr(), sv[1, t].data_ptr(), sv[2, t].data_ptr(), sv[3, t].data_ptr(),
                                    sv[4, t].data_ptr(), hd, N, hd, st)
            if rc:
                raise RuntimeError('mfg_gru_fwd_step failed')
            lo += 3 * hd

    def _sample(self, logits, t):
        """a_t ~ Categorical(logits) per agent into act[t] (base_ac.py:74-76): on the GPU one kernel
        (mfg_sample_categorical) on uniforms drawn into a static buffer; an explicit generator keeps
        torch.multinomial."""
        if self.gen is not None:
            a = torch.multinomial(torch.softmax(logits, -1), 1, generator=self.gen).squeeze(-1)
            self.act[t].copy_(a.view(self.B, self.A))
            return
        if not logits.is_cuda:
            self.act[t].copy_(Categorical(logits=logits, validate_args=False).sample().view(self.B, self.A))
            return
        logits = logits.contiguous()
        self._u.uniform_()
        rc = _gru_lib().mfg_sample_categorical(logits.data_ptr(), logits.stride(0), logits.shape[1],
                                               self._u.data_ptr(), self.N, self.act[t].data_ptr(),
                                               torch.cuda.current_stream(self.dev).cuda_stream)
        if rc:
            raise RuntimeError('mfg_sample_categorical failed')

    def _policy_step(self, t):
        if not self.act_graph:
            return self._policy(t)
        g = self._act_graphs.get(t)
        if g is not None:
            g.replay()
            return
        cur = torch.cuda.current_stream(self.dev)
        if self._act_warm.get(t, 0) < 2:  # eager warm-up on a side stream (lazy library state outside the capture)
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self._policy(t)
            cur.wait_stream(side)
            self._act_warm[t] = self._act_warm.get(t, 0) + 1
            return
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._policy(t)
        self._act_graphs[t] = g
        g.replay()  # capture records only: this step's policy runs here

    def window(self):
        """The window's learner inputs: packed entries [N, T+1, cap], action inputs [N, T+1], starts,
        targets."""
        T, N = self.T, self.N
        idx = self.pobs.idx.permute(1, 2, 0, 3).reshape(N, T + 1, -1)
        val = self.pobs.val.permute(1, 2, 0, 3).reshape(N, T + 1, -1)
        a_in = self.act_in.permute(1, 2, 0).reshape(N, T + 1)
        acts = torch.cat([a_in[:, :1], self.act.permute(1, 2, 0).reshape(N, T).long()], 1)
        d = self.done.permute(1, 0).repeat_interleave(self.A, 0).to(torch.float32)  # [N, T]
        starts = torch.cat([torch.zeros((N, 1), dtype=torch.bool, device=self.dev), d.bool()], 1)
        rew = self.rew.permute(1, 2, 0).reshape(N, T).to(torch.float32)
        return idx, val, a_in, acts, starts, rew, d

    def loss(self):
        """The A2C loss of the current window (base_ac.py:200-217), with grad."""
        if self.reuse:
            return self._loss_saved()
        return self._loss_recompute()

    def _loss_saved(self):
        """loss() from the acting steps' stored forward (reuse_acting), entry-major rows (t, n): obs_proj through
        _EngineProj on the window's packed rows in place, the mix through _MixSaved and the GRUs through
        _GRUWindowSavedT (stored forwards, backward only), the heads with grad; the entry-T critic (the bootstrap
        target, detached in base_ac.py:185-198) by one no-grad step from the carried state."""
        T, N, cap, A = self.T, self.N, self.pobs.cap, self.A
        net = self.net
        rows = T * N
        d = self.done.to(torch.float32).repeat_interleave(A, 1)  # [T, N]: done after entry t
        keep = torch.ones((T, N), dtype=torch.float32, device=self.dev)
        keep[1:] = 1.0 - d[:-1]  # entry s > 0 restarts after an episode end at s - 1
        with torch.no_grad():
            xT = net.mixed(self.pobs.emb[T].view(N, 1, -1), self.act_in[T].view(N, 1), self.agent_ids)[:, 0]
            gc = net.gru_critic
            hT = torch.gru_cell(xT, self.hc[:, 0], gc.weight_ih_l0, gc.weight_hh_l0, gc.bias_ih_l0, gc.bias_hh_l0)
            critic_T = net.critic_head(hT)  # [N, 1]
        with torch.enable_grad():
            idx, val = self.pobs.idx[:T].reshape(rows, cap), self.pobs.val[:T].reshape(rows, cap)
            if self.engine_emb:
                emb = _EngineProj.apply(idx, val, net.obs_proj.weight, net.obs_proj.bias,
                                        self.pobs.emb[:T].reshape(rows, -1))
            else:
                emb = net.project_packed(idx, val)
            mixed = _MixSaved.apply(emb, net.mix[1].weight, net.mix[1].bias, net.mix[3].weight, net.mix[3].bias,
                                    net.action_emb.weight, (self.ax.view(rows, -1), self.h1.view(rows, -1),
                                                            self.mx.view(rows, -1), self.act_in[:T].reshape(rows),
                                                            net.action_emb.padding_idx))
            ga, gc = net.gru_actor, net.gru_critic
            out_p, out_c = _GRUWindowSavedT.apply(mixed, keep, (self.hs_a, self.hs_c, self.sv_a, self.sv_c),
                                                  ga.weight_ih_l0, ga.weight_hh_l0, ga.bias_ih_l0, ga.bias_hh_l0,
                                                  gc.weight_ih_l0, gc.weight_hh_l0, gc.bias_ih_l0, gc.bias_hh_l0)
            out = net._heads(out_p, out_c, True)
            logits = out['logits'].view(T, N, -1).transpose(0, 1)  # [N, T, n_act]
            critic = torch.cat([out['critic'].view(T, N).t(), critic_T], 1)  # [N, T + 1]
            acts = torch.cat([self.act_in[0].reshape(N, 1), self.act.reshape(T, N).t().long()], 1)
            rew = self.rew.reshape(T, N).t().to(torch.float32)
            return a2c_loss_terms(logits, critic, acts, rew, d.t(), self.gamma, self.entropy_coef, self.vf_coef,
                                  self.gae_coef)

    def _loss_recompute(self):
        """loss() with the whole window's forward recomputed (the reference learner's order, base_ac.py:126-128)."""
        idx, val, a_in, acts, starts, rew, d = self.window()
        with torch.enable_grad():
            if self.engine_emb:  # the forward from the render's fused projection (same weights), no gather
                T, N, cap = self.T, self.N, idx.shape[-1]
                emb_pre = self.pobs.emb.permute(1, 2, 0, 3).reshape(N * (T + 1), -1)
                emb = _EngineProj.apply(idx.reshape(-1, cap), val.reshape(-1, cap), self.net.obs_proj.weight,
                                        self.net.obs_proj.bias, emb_pre).view(N, T + 1, -1)
            else:
                emb = self.net.project_packed(idx, val)
            out = self.net.forward_emb(emb, a_in, self.h0a, self.h0c, agent_ids=self.agent_ids, starts=starts)
            return a2c_loss(out, acts, rew, d, self.gamma, self.entropy_coef, self.vf_coef, self.gae_coef)

    def learn(self):
        """One A2C update on the window (base_ac.py:200-225), then slide: o_T becomes o_0."""
        if self.check_cap:
            self.pobs.check()
            if self.gen is None and self.dev.type == 'cuda' and bool((self.act < 0).any()):
                # mfg_sample_categorical marks rows with non-finite logits -1 (the engine took them as crash actions)
                raise RuntimeError('BatchedA2C: non-finite policy logits in this window (training diverged)')
        # episode and reward counters once per window (two reductions instead of two per step)
        self.episodes += self.done.sum()
        self.reward_sum += self.rew.sum()
        if not self.graph:
            self._update()
        elif self._graph is not None:
            self._graph.replay()
        elif self._warm < 2:  # eager warm-up on a side stream (lazy library state outside the capture)
            side = torch.cuda.Stream(self.dev)
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):
                self._update()
            torch.cuda.current_stream(self.dev).wait_stream(side)
            self._warm += 1
        else:
            g = torch.cuda.CUDAGraph()
            self.opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(g):
                self._update()
            self._graph = g
            g.replay()  # capture records only: this update runs here
        self.updates += 1
        self.t = 0

    def _update(self):
        """The update and the slide on static buffers (the body HIP-graph captured when graph=True)."""
        with torch.enable_grad():
            loss = self.loss()
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(self.net.parameters(), 0.5)
            self.opt.step()
        with torch.no_grad():
            self.last_loss.copy_(loss.detach())
            T = self.T
            self.pobs.idx[0].copy_(self.pobs.idx[T])
            self.pobs.val[0].copy_(self.pobs.val[T])
            self.pobs.count[0].copy_(self.pobs.count[T])
            self.act_in[0].copy_(self.act_in[T])
            self.h0a.copy_(self.ha)
            self.h0c.copy_(self.hc)
            # new weights: the engine projects with them from now on; o_0's projection is redone here
            self.pobs.set_projection(self.net.obs_proj.weight, self.net.obs_proj.bias)
            self._project_slot0()

    def _project_slot0(self):
        """o_0's fused projection redone with the new weights (the engine rendered it with the old ones): one
        mfg_packed_project over its packed rows on the GPU."""
        pb = self.pobs
        if not pb.idx.is_cuda:
            pb.emb[0].copy_(_project_dense(pb.idx[0], pb.val[0], self.net.obs_proj))
            return
        rc = _gru_lib().mfg_packed_project(pb.idx[0].data_ptr(), pb.val[0].data_ptr(), self.N, pb.cap, pb.wt.data_ptr(),
                                           pb.bias.data_ptr(), pb.E, pb.kdim, pb.emb[0].data_ptr(), pb.E,
                                           torch.cuda.current_stream(self.dev).cuda_stream)
        if rc:
            raise RuntimeError('mfg_packed_project failed')

    def train(self, n_updates):
        for _ in range(n_updates * self.T):
            self.step()
        return self.last_loss
