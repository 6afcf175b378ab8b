# one-off check of parallel.gather_distinct_flows on one GPU (world 1, gloo): sizes at each stage
import socket, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "net-parser-rs_amd")
import torch, torch.distributed as dist
from net_parser_rs import parallel, device, synth
import test_gpu_flowtable as t
blob = synth.flow_mix(30_000, n_flows=700, seed=12)
fl, f6, n = t.device_table(blob)
print("n", n, fl.shape, f6.shape, fl.device)
r = parallel.device_aggregate(fl[: n * 32], f6[: n * 32], n)
print("local k", r[3], r[0].shape, r[2][:5])
r2 = parallel.device_aggregate(r[0].contiguous(), r[1].contiguous(), r[3], r[2].contiguous())
print("merge of local k", r2[3], r2[2][:5])
rc = [x.cpu() if torch.is_tensor(x) else x for x in r]
r3 = parallel.device_aggregate(rc[0].cuda(), rc[1].cuda(), r[3], rc[2].cuda())
print("merge via host k", r3[3])
s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
g = parallel.gather_distinct_flows(fl[: n * 32], f6[: n * 32], n)
print("gather k", g[3])
dist.destroy_process_group()
