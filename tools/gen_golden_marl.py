#!/usr/bin/env python3
"""Golden vectors for the A2C learner: runs the REFERENCE network and loss
(algorithms/marl/networks.py RecurrentAC, algorithms/marl/base_ac.py actor_critic + learn) on a small
synthetic memory and stores inputs, weights, loss, gradients and the weights after one RMSprop step.

THIS SCRIPT RUNS ONLY IN THE DEVELOPMENT CONTAINER (it imports /root/reference read-only). Output:
tests/golden/marl_a2c.npz (data only). tests/test_marl.py replays it through mfg_amd.marl on packed obs.
"""
import sys
import types
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / 'tools' / 'standins'), '/root/reference']

from marl_factory_grid.algorithms.marl.networks import RecurrentAC  # noqa: E402
from marl_factory_grid.algorithms.marl.base_ac import BaseActorCritic  # noqa: E402

VALUES = np.array([1.0, 2.0, 0.6666, 0.4444, 0.37, 3.0])


def case(seed, gae_coef, use_agent_embedding):
    rng = np.random.default_rng(seed)
    N, T, L, d, n_actions = 2 if use_agent_embedding else 6, 5, 4, 5, 10
    obs = np.zeros((N, T + 1, L, d, d))
    mask = rng.random(obs.shape) < 0.06
    obs[mask] = rng.choice(VALUES, mask.sum())
    actions = rng.integers(0, n_actions, (N, T + 1))
    actions[:, 0] = rng.choice([-1, 3], N)
    reward = rng.normal(0, 0.3, (N, T + 1)).astype(np.float32)
    done = (rng.random((N, T + 1)) < 0.15).astype(np.float32)
    ha = rng.normal(0, 0.5, (N, T + 1, 1, 32)).astype(np.float32)
    hc = rng.normal(0, 0.5, (N, T + 1, 1, 32)).astype(np.float32)
    torch.manual_seed(seed)
    net = RecurrentAC(observation_size=(L, d, d), n_actions=n_actions, obs_emb_size=40, action_emb_size=8,
                      hidden_size_actor=32, hidden_size_critic=32, n_agents=N,
                      use_agent_embedding=use_agent_embedding)
    state = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}
    tm = types.SimpleNamespace(observation=torch.from_numpy(obs), action=torch.from_numpy(actions),
                               done=torch.from_numpy(done), reward=torch.from_numpy(reward),
                               hidden_actor=torch.from_numpy(ha), hidden_critic=torch.from_numpy(hc))
    owner = types.SimpleNamespace(compute_advantages=BaseActorCritic.compute_advantages)
    loss = BaseActorCritic.actor_critic(owner, tm, net, gamma=0.99, entropy_coef=0.01, vf_coef=0.5,
                                        gae_coef=gae_coef)
    opt = torch.optim.RMSprop(net.parameters(), lr=3e-4, eps=1e-5)  # base_ac.py:47
    opt.zero_grad()
    loss.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().numpy().copy()
             for k, p in net.named_parameters()}
    torch.nn.utils.clip_grad_norm_(net.parameters(), 0.5)  # base_ac.py:224
    opt.step()
    after = {k: p.detach().numpy().copy() for k, p in net.named_parameters()}
    out = {'obs': obs, 'actions': actions, 'reward': reward, 'done': done, 'ha0': ha[:, 0], 'hc0': hc[:, 0],
           'loss': np.float64(loss.item()), 'gae_coef': np.float64(gae_coef),
           'use_agent_embedding': np.int32(use_agent_embedding), 'n_actions': np.int32(n_actions)}
    for k, v in state.items():
        out['w.' + k] = v
    for k, v in grads.items():
        out['g.' + k] = v
    for k, v in after.items():
        out['a.' + k] = v
    return out


def main():
    res = {}
    for i, (seed, gae, ae) in enumerate([(0, 0.0, False), (1, 0.95, False), (2, 0.0, True)]):
        for k, v in case(seed, gae, ae).items():
            res[f'c{i}.{k}'] = v
    dst = REPO / 'tests' / 'golden' / 'marl_a2c.npz'
    np.savez_compressed(dst, **res)
    print('wrote', dst, dst.stat().st_size, 'bytes')


if __name__ == '__main__':
    main()
