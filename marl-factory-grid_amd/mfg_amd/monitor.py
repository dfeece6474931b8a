"""Episode monitoring and state recording over the facade (utils/logging/).

* `EnvMonitor` -- utils/logging/envmonitor.py:14-73: wraps a `Factory`, keeps every step's info dict
  and, at each done, aggregates the episode (columns ending in 'ount' averaged, the others summed,
  IGNORED_DF_COLUMNS dropped, helpers.py:26-28) into one DataFrame row; `save_monitor` pickles the
  DataFrame (our own file, written the way the reference writes it); `auto_plotting_keys` plots the saved
  file with `mfg_amd.plotting.plot_single_run` (utils/plotting/plot_single_runs.py).
* `EnvRecorder` -- utils/logging/recorder.py:10-190: records `summarize_state()` per step for the chosen
  episodes and writes them with the reference's record layout ({'episodes': [{'steps', 'episode_nr'}],
  'n_episodes', 'metadata', 'header'}). The reference serialises that dict through a generated protobuf
  module (utils/proto/fiksProto_pb2), which is not part of this build: records are written as JSON.
  `only_deltas` writes the differences between consecutive episodes (DeepDiff when importable, else a
  built-in structural diff with DeepDiff's report keys); `save_occupation_map` writes the agents' cell-visit
  counts over the level (.npy, plus a .png heatmap when matplotlib is importable; the reference sums into a
  fixed 15x15 array from a key its summary does not have, recorder.py:171-187); `save_trajectory_map` raises
  NotImplementedError like the reference (recorder.py:189-190).
* `BatchedEpisodeLog` -- the batched counterpart: per-episode returns/lengths of a `VectorFactory`,
  collected from its step infos without per-step host copies of the whole batch.
"""
import json
import pickle
from pathlib import Path

IGNORED_DF_COLUMNS = ['Episode', 'Run', 'train_step', 'step', 'index', 'dirt_amount', 'dirty_pos_count',
                      'terminal_observation', 'episode']


class _Wrapper:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        return getattr(self.env, name)


class EnvMonitor(_Wrapper):
    ext = 'png'

    def __init__(self, env, filepath=None):
        super().__init__(env)
        import pandas as pd
        self._pd = pd
        self._filepath = filepath
        self._monitor_df = pd.DataFrame()
        self._monitor_dict = dict()

    def step(self, action):
        obs_type, obs, reward, done, info = self.env.step(action)
        self._read_info(info)
        self._read_done(done)
        return obs_type, obs, reward, done, info

    def reset(self):
        return self.env.reset()

    def _read_info(self, info):
        self._monitor_dict[len(self._monitor_dict)] = {k: v for k, v in info.items()
                                                       if k not in ['terminal_observation', 'episode']}

    def _read_done(self, done):
        if not done:
            return
        pd = self._pd
        df = pd.DataFrame.from_dict(self._monitor_dict, orient='index')
        self._monitor_dict = dict()
        columns = [c for c in df.columns if c not in IGNORED_DF_COLUMNS]
        agg = df.aggregate({c: 'mean' if c.endswith('ount') else 'sum' for c in columns})
        agg['episode'] = len(self._monitor_df)
        self._monitor_df = pd.concat([self._monitor_df, pd.DataFrame([agg])], ignore_index=True)

    @property
    def monitor_df(self):
        return self._monitor_df

    def save_monitor(self, filepath=None, auto_plotting_keys=None):
        filepath = Path(filepath or self._filepath)
        filepath.parent.mkdir(exist_ok=True, parents=True)
        with filepath.open('wb') as f:
            pickle.dump(self._monitor_df.reset_index(), f, protocol=pickle.HIGHEST_PROTOCOL)
        if auto_plotting_keys:
            from .plotting import plot_single_run
            plot_single_run(filepath, column_keys=auto_plotting_keys)

    def report_possible_colum_keys(self):
        print(self._monitor_df.columns)


class EnvRecorder(_Wrapper):
    def __init__(self, env, filepath=None, episodes=None):
        super().__init__(env)
        self.filepath = filepath
        self.episodes = episodes
        self._curr_episode = 0
        self._curr_ep_recorder = list()
        self._recorder_out_list = list()

    def reset(self):
        self._curr_ep_recorder = list()
        self._recorder_out_list = list()
        self._curr_episode += 1
        return self.env.reset()

    def step(self, actions):
        obs_type, obs, reward, done, info = self.env.step(actions)
        if not self.episodes or self._curr_episode in self.episodes:
            self._curr_ep_recorder.append(self.env.summarize_state())
            if done:
                self._recorder_out_list.append({'steps': self._curr_ep_recorder, 'episode_nr': self._curr_episode})
                self._curr_ep_recorder = list()
        return obs_type, obs, reward, done, info

    def _finalize(self):
        if self._curr_ep_recorder:
            self._recorder_out_list.append({'steps': self._curr_ep_recorder.copy(),
                                            'episode_nr': len(self._recorder_out_list)})

    def records(self):
        """The record dict save_records writes (recorder.py:96-158 layout)."""
        params = self.env.params
        return {'episodes': self._recorder_out_list, 'n_episodes': self._curr_episode,
                'metadata': dict(level_name=params['General']['level_name'], n_agents=len(params['Agents']),
                                 env_seed=params['General'].get('env_seed', 69),
                                 pomdp_r=params['General']['pomdp_r'], individual_rewards=True),
                'header': self.env.summarize_header()}

    def save_records(self, filepath=None, only_deltas=False, save_occupation_map=False, save_trajectory_map=False):
        self._finalize()
        filepath = Path(filepath or self.filepath)
        filepath.parent.mkdir(exist_ok=True, parents=True)
        rec = self.records()
        if only_deltas:
            eps = rec['episodes']
            rec['episodes'] = [_deltas(a, b) for a, b in zip(eps, eps[1:])]
        with filepath.open('w') as f:
            json.dump(rec, f, default=str)
        if save_occupation_map:
            self.occupation_map(filepath.with_name(filepath.stem + '_occupation'))
        if save_trajectory_map:
            raise NotImplementedError('This has not yet been implemented.')  # as the reference (recorder.py:189-190)
        return filepath

    def occupation_map(self, out_stem=None):
        """[H, W] counts of agent positions over every recorded step (recorder.py:171-180, over the level's
        shape); with out_stem, written to <out_stem>.npy and, if matplotlib is importable, <out_stem>.png."""
        import numpy as np
        H, W = self.env.spec.H, self.env.spec.W
        occ = np.zeros((H, W), np.int64)
        for ep in self._recorder_out_list:
            for st in ep['steps']:
                for a in st.get('agents', []):
                    if 0 <= a['x'] < H and 0 <= a['y'] < W:
                        occ[a['x'], a['y']] += 1
        if out_stem is not None:
            out_stem = Path(out_stem)
            np.save(out_stem.with_suffix('.npy'), occ)
            try:
                import matplotlib
                matplotlib.use('Agg')
                import matplotlib.pyplot as plt
            except Exception:
                return occ
            fig, ax = plt.subplots(figsize=(6, 6 * H / max(W, 1) + 0.5))
            im = ax.imshow(occ, cmap='viridis')
            fig.colorbar(im, ax=ax)
            ax.set_title('agent occupation')
            fig.savefig(out_stem.with_suffix('.png'))
            plt.close(fig)
        return occ


def _deltas(t1, t2):
    """Differences between two episode records: DeepDiff(t1, t2, ignore_order=True) (recorder.py:91-95) when
    deepdiff is importable, else a structural diff reporting DeepDiff's keys for ordered data
    (values_changed, type_changes, dictionary_item_added/removed, iterable_item_added/removed)."""
    try:
        from deepdiff import DeepDiff
        return json.loads(DeepDiff(t1, t2, ignore_order=True).to_json())
    except ImportError:
        pass
    out = {}

    def put(kind, path, val):
        out.setdefault(kind, {})[path] = val

    def walk(a, b, path):
        if isinstance(a, dict) and isinstance(b, dict):
            for k in a:
                if k not in b:
                    put('dictionary_item_removed', f"{path}['{k}']", a[k])
                else:
                    walk(a[k], b[k], f"{path}['{k}']")
            for k in b:
                if k not in a:
                    put('dictionary_item_added', f"{path}['{k}']", b[k])
        elif isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
            for i in range(min(len(a), len(b))):
                walk(a[i], b[i], f'{path}[{i}]')
            for i in range(len(b), len(a)):
                put('iterable_item_removed', f'{path}[{i}]', a[i])
            for i in range(len(a), len(b)):
                put('iterable_item_added', f'{path}[{i}]', b[i])
        elif type(a) is not type(b):
            put('type_changes', path, {'old_type': type(a).__name__, 'new_type': type(b).__name__,
                                       'old_value': a, 'new_value': b})
        elif a != b:
            put('values_changed', path, {'old_value': a, 'new_value': b})

    walk(t1, t2, 'root')
    return out


class BatchedEpisodeLog:
    """Finished-episode statistics of a `VectorFactory`: call `update(infos)` after each step."""

    def __init__(self):
        self.returns, self.lengths, self.env_ids = [], [], []

    def update(self, infos):
        if '_final' not in infos:
            return 0
        idx = infos['_final'].nonzero().flatten()
        if idx.numel() == 0:
            return 0
        self.returns.append(infos['final_return'][idx].cpu())
        self.lengths.append(infos['final_length'][idx].cpu())
        self.env_ids.append(idx.cpu())
        return int(idx.numel())

    def frame(self):
        import pandas as pd
        import torch
        if not self.returns:
            return pd.DataFrame(columns=['env', 'length', 'return_sum'])
        r = torch.cat(self.returns)
        df = pd.DataFrame({'env': torch.cat(self.env_ids).numpy(), 'length': torch.cat(self.lengths).numpy(),
                           'return_sum': r.sum(dim=1).numpy()})
        for a in range(r.shape[1]):
            df[f'return_{a}'] = r[:, a].numpy()
        return df
