cd $GRAFT_REPO_ROOT
for w in 4 2 1; do
MFG_REPLAY_WPB=$w timeout -k 10 300 python bench.py --steps 400 --warmup 100 --no-cpu-baseline --alt-steps 0 --packed-steps 0 | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['roofline'].get('kernels',{})
print('wpb $w', d['value'], {n: v['mean_launch_ms'] for n, v in k.items()})" || exit 1
done
