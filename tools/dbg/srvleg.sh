python -u -c "
import json, torch, bench
d = torch.device('cuda:0'); torch.cuda.set_device(d)
r = bench.server_group_leg(d, 1, 0)
print(json.dumps({k: r[k] for k in ('node_GiBps', 'round_ms', 'copying_pulls', 'exact_vs_torch_sum')}))
"
