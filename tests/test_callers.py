"""Callers drop in (SURVEY §8(b) 'Callers'): the reference's example script random_testrun.py imports
  marl_factory_grid.environment.factory.Factory, marl_factory_grid.utils.logging.{envmonitor,recorder},
  marl_factory_grid.utils.plotting.plot_single_runs.plot_single_run, marl_factory_grid.utils.tools.ConfigExplainer
and runs configs/eight_puzzle.yaml with random actions until done, 10 episodes, then saves and plots the
monitor (random_testrun.py:1-66). CPU: every import path resolves through the compat package and the host-only
pieces work. GPU: the same loop on the engine."""
import random
import sys
from pathlib import Path

import pytest

from conftest import gpu_available

ROOT = Path(__file__).resolve().parent.parent
COMPAT = ROOT / 'marl-factory-grid_amd' / 'compat'


@pytest.fixture
def compat_path(monkeypatch):
    monkeypatch.syspath_prepend(str(COMPAT))
    yield


def test_compat_import_paths(compat_path):
    from marl_factory_grid.environment.factory import Factory
    from marl_factory_grid.utils.logging.envmonitor import EnvMonitor
    from marl_factory_grid.utils.logging.recorder import EnvRecorder
    from marl_factory_grid.utils.plotting.plot_single_runs import plot_single_run
    from marl_factory_grid.utils.tools import ConfigExplainer
    import mfg_amd.factory as F
    import mfg_amd.monitor as M
    assert Factory is F.Factory and EnvMonitor is M.EnvMonitor and EnvRecorder is M.EnvRecorder
    assert callable(plot_single_run) and callable(ConfigExplainer().save_all)


def test_config_explainer_lists_what_compiles(tmp_path, compat_path):
    """Every class the explainer lists is one the spec compiler maps onto the engine."""
    import yaml
    from marl_factory_grid.utils.tools import ConfigExplainer
    from mfg_amd import spec as S
    ce = ConfigExplainer()
    out = ce.save_all(tmp_path / 'study_out' / 'all_available_configs.yaml')
    data = yaml.safe_load(out.read_text())
    assert set(data) == {'General', 'Agents', 'Entities', 'Rules'}
    assert set(data['Entities']) == set(S._GROUPS)
    assert set(data['Rules']) == set(S._RULES) | set(S._DEST_SPAWNRULES)
    assert set(ce.get_actions()) == set(S._ACTIONS) | set(S._MOVE_GROUPS)


def test_config_explainer_lists_custom_rules(compat_path):
    """utils/tools.py:24-39: a custom path adds its Rule classes (explained by their __init__ defaults); they
    run on the host beside the engine (custom_modules_path)."""
    from pathlib import Path
    from marl_factory_grid.utils.tools import ConfigExplainer
    from mfg_amd import spec as S
    rules = ConfigExplainer(Path(__file__).parent / 'custom_rules').get_rules()
    assert rules['DoneWhenCrowded'] == {'k': 3, 'reward': -1.0}
    assert rules['DoorProximityBonus'] == {'bonus': 0.05}
    assert set(rules) == set(S._RULES) | set(S._DEST_SPAWNRULES) | {
        'DoorProximityBonus', 'CountFailedActions', 'PenaltyBeforeActions', 'DoneWhenCrowded'}


def test_plot_single_run_from_monitor_file(tmp_path):
    import pandas as pd
    import pickle
    from mfg_amd.plotting import plot_single_run
    df = pd.DataFrame({'step_reward': [1.0, -0.5, 2.0], 'Agent[W]_Noop': [0.1, 0.2, None], 'step': [3, 4, 5]})
    with (tmp_path / 'test_monitor.pkl').open('wb') as f:
        pickle.dump(df, f)
    out = plot_single_run(tmp_path, column_keys=['step_reward'])
    assert out.exists() and out.stat().st_size > 0


@pytest.mark.gpu
def test_random_testrun_loop_on_the_engine(tmp_path, monkeypatch, compat_path):
    """random_testrun.py's body with monitor=True, record=True, plotting=True, through the compat imports."""
    if not gpu_available():
        pytest.skip('no GPU')
    from marl_factory_grid.environment.factory import Factory
    from marl_factory_grid.utils.logging.envmonitor import EnvMonitor
    from marl_factory_grid.utils.logging.recorder import EnvRecorder
    from marl_factory_grid.utils.plotting.plot_single_runs import plot_single_run
    from marl_factory_grid.utils.tools import ConfigExplainer
    monkeypatch.chdir(tmp_path)
    run_path = Path('study_out')
    ConfigExplainer().save_all(run_path / 'all_available_configs.yaml')
    factory = Factory(Path('marl_factory_grid/configs/eight_puzzle.yaml'))  # resolved by config name
    factory = EnvMonitor(factory)
    factory = EnvRecorder(factory)
    random.seed(5)
    episodes_done = 0
    for episode in range(10):
        _ = factory.reset()
        done = False
        action_spaces = factory.action_space
        steps = 0
        while not done:
            a = [random.randint(0, x.n - 1) for x in action_spaces]
            obs_type, obs, reward, done, info = factory.step(a)
            steps += 1
            assert len(obs) == 8 and obs[0].shape == (9, 5, 5)  # 7 Other + Walls + Destination over the 5x5 level
            assert isinstance(info, dict) and info['step'] == steps
            if done:
                episodes_done += 1
                break
        assert steps <= 200
    factory.save_monitor(run_path / 'test_monitor.pkl')
    factory.save_records(run_path / 'test.pb')
    factory.report_possible_colum_keys()
    plot_single_run(run_path, column_keys=['step_reward'])
    assert episodes_done == 10
    assert (run_path / 'test_monitor.pkl').exists() and any(run_path.glob('test_monitor.*'))
