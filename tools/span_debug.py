"""Debug aid for the route-all span mode: lifted-cap frames verify over an aligned
dense stream; prints every body whose CRC differs from the oracle's."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import rpc_amd  # noqa: E402
from oracle import oracle  # noqa: E402

HDR = 12
DEV = "cuda:0"
rng = np.random.default_rng(5)
lens = [1, 5, 4083, 4084, 4085, 4096 - HDR, 8192, 8193, 12288 - 7, 3 << 20, 77, 65536 + 3, 4096, 4095, 2, 40000]
lens += rng.integers(0, 20000, 20).tolist()
sizes = [HDR + L for L in lens]
total = sum(sizes)
t = torch.empty(total + 8192, dtype=torch.uint8, device=DEV)
off = (-t.data_ptr()) % 4096
base = t[off:off + total]
fill = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=DEV)
rpc_amd.fill_random(fill, 0x77)
base.copy_(fill[:total])
offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
do = torch.from_numpy(offs.view(np.int64)).to(DEV)
dl = torch.from_numpy(np.array(lens, dtype=np.uint32).view(np.int32)).to(DEV)
sv = rpc_amd.frames_stamp(base, do, dl, lift_cap=True, stream_bytes=total)
print("stamp verdicts", sv.cpu().numpy().tolist())
host = base.cpu().numpy()
c = np.array([int.from_bytes(host[int(o) + 8:int(o) + 12].tobytes(), "big") for o in offs], dtype=np.uint32)
bad = 0
for i, (o, L) in enumerate(zip(offs, lens)):
    s = int(o) + HDR
    want = oracle.crc32(host[s:s + L])
    if int(c[i]) != want:
        bad += 1
        e = s + L
        j0, j1 = s >> 12, (e - 1) >> 12
        print(f"body {i}: s={s} (s&4095={s & 4095}) L={L} e&4095={e & 4095} nch={j1 - j0 + 1} got={int(c[i]):08x} want={want:08x}")
print(f"{bad} of {len(lens)} bodies wrong; total {total}; base aligned {base.data_ptr() % 4096 == 0}")
