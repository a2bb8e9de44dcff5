import sys, types
import numpy as np, torch
sys.argv = ["bench.py", "--workload", "hetero", "--hetero-n", "64", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
sys.path.insert(0, "."); import bench
orig = torch.Tensor.copy_
def spy(self, src, *a, **k):
    r = orig(self, src, *a, **k)
    if self.dtype == torch.int32 and self.dim() == 1:
        torch.cuda.synchronize()
        s = src.cpu().numpy().view(np.uint32); d = self.cpu().numpy().view(np.uint32)
        print("copy src", float(((s & 1) > 0).mean()), "nz", int((s != 0).sum()), "dst nz", int((d != 0).sum()), flush=True)
    return r
torch.Tensor.copy_ = spy
bench.main()
