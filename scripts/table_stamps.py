"""Phase clocks of the device table build (a -DMH_TABLE_STAMPS=1 library via MH_LIB):
s_memtime after each barrier of workgroup 0, stored past the prepared table."""
import sys

import torch

sys.path.insert(0, ".")
import metalhuffman_amd as mh  # noqa: E402
from metalhuffman_amd import decoder as D  # noqa: E402
from metalhuffman_amd import frames as F  # noqa: E402
from metalhuffman_amd import _native as N  # noqa: E402

canon = mh.encode_frame(F.bigbridge()).canon
dev = torch.device("cuda:0")
for _ in range(3):
    tabs = D.DeviceTables.from_canonical_header(canon, dev)
    torch.cuda.synchronize()
    base = int(N.lib().mh_lut_bytes()) - 256
    st = tabs.lut[base: base + 128].cpu().view(torch.int64).tolist()
    n = max(i for i, v in enumerate(st) if v)
    print("phase clocks:", [st[i + 1] - st[i] if st[i + 1] and st[i] else None for i in range(n)],
          "total", st[n] - st[0])
