"""host_inclusive (bench.py) over sub-batch counts and size-readback modes (GPU box)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..'))
import numpy as np
import torch

import bench
from wanproxy_amd import synth
from wanproxy_amd.xcgpu import Context

dev = torch.device('cuda', 0)
n, CH = 4096, 65536
data = np.frombuffer(synth.stream(0xC2, n * CH, 50, 0), np.uint8)
offs, lens = synth.chunks_of(data.tobytes(), CH)
bounds = 2 * lens.astype(np.uint64) + 16
oo = np.zeros(n, np.uint64)
oo[1:] = np.cumsum(bounds)[:-1]
d_in = torch.from_numpy(data.copy()).to(dev)
d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
d_oo = torch.from_numpy(oo.view(np.int64)).to(dev)
d_out = torch.empty(int(bounds.sum()), dtype=torch.uint8, device=dev)
d_ol = torch.zeros(n, dtype=torch.int64, device=dev)
ctx = Context(0)
for zc in (False, True):
    for nsub in [int(v) for v in os.environ.get("NSUBS", "8,16,32,64").split(",")]:
        r = bench.host_inclusive(ctx, data, offs, lens, d_in, d_off, d_len, d_oo, d_out, d_ol, n, dev, nsub=nsub,
                                 zero_copy=zc)
        print(json.dumps({'zero_copy': zc, 'nsub': nsub, 'GiBps': r['value'], 'pcie_GBps': r['pcie_GBps']}), flush=True)
