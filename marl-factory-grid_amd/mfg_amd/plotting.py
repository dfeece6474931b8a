"""Per-run reward curves from an EnvMonitor file (the reference's utils/plotting/plot_single_runs.py:12-70).

Reads the pickled monitor DataFrame our own EnvMonitor.save_monitor wrote, keeps the requested columns
(all but the ignored ones by default) per episode, and writes `<monitor stem>.png` with matplotlib, or a CSV
of the same series when matplotlib is not importable.
"""
import pickle
from pathlib import Path

from .monitor import IGNORED_DF_COLUMNS


def plot_single_run(run_path, use_tex=False, column_keys=None, file_key='monitor', file_ext='pkl'):
    run_path = Path(run_path)
    if run_path.is_dir():
        monitor_file = next(run_path.glob(f'*{file_key}*.{file_ext}'))
    elif run_path.is_file():
        monitor_file = run_path
    else:
        raise ValueError(f'no monitor file at {run_path}')
    with monitor_file.open('rb') as f:  # a file this package wrote (EnvMonitor.save_monitor)
        df = pickle.load(f).fillna(0)
    cols = [c for c in df.columns if c not in IGNORED_DF_COLUMNS] if column_keys is None else \
        [c for c in column_keys if c in df.columns]
    series = df[cols]
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
    except Exception:
        out = monitor_file.with_suffix('.csv')
        series.to_csv(out)
        return out
    fig, ax = plt.subplots(figsize=(6, 3.5))
    for c in cols:
        ax.plot(series.index, series[c], label=c)
    ax.set_xlabel('episode')
    ax.set_ylabel('value')
    ax.legend(fontsize=7)
    fig.tight_layout()
    out = monitor_file.with_suffix('.png')
    fig.savefig(out)
    plt.close(fig)
    return out
