import sys, time, torch
sys.path.insert(0, ".")
import metalhuffman_amd as mh
from metalhuffman_amd import decoder as D, frames as F
ef = mh.encode_frame(F.bigbridge()); t1, t2 = ef.tables()
dev = torch.device("cuda:0")
tabs = D.DeviceTables.upload(t1, t2, dev); torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    for _ in range(100): tabs.prepare_lut()
    torch.cuda.synchronize(); print(f"mh_prepare_lut {1e6*(time.perf_counter()-t0)/100:.1f} us")
