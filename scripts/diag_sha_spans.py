"""Diagnostic: cycles per SHA-256 round of k_sha256 on controlled span layouts
(one long span per workgroup vs full workgroups), product mode and diag modes."""
import os
os.environ["CHUNKER_AMD_DIAG"] = "1"  # load libchunker_amd_diag.so (make -C chunker_amd/csrc diag)
os.environ.setdefault("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR", "1")
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import chunker_amd as ca  # noqa: E402

lib = ca.lib
lib.cg_diag_sha_stats.argtypes = [ctypes.c_uint32, ctypes.c_void_p]
lib.cg_diag_sha_mode.argtypes = [ctypes.c_uint32]
lib.cg_hash_spans_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
BIG = 4 << 20
data = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device="cuda")
layouts = {
    "1span": [BIG],
    "64lanes_1wg": [BIG] * 64,
    "16wg_1lane": [BIG if i % 64 == 0 else 64 for i in range(1024)],
    "16wg_full": [BIG] * 1024,
    "128wg_1lane": [BIG if i % 64 == 0 else 64 for i in range(8192)],
}
res = {}
modes = [int(m) for m in sys.argv[1:]] or [0, 2]
for name, lens in layouts.items():
    n = len(lens)
    lens_t = torch.tensor(lens, dtype=torch.int64, device="cuda")
    offs_t = (torch.arange(n, dtype=torch.int64, device="cuda") * 4099) % (60 << 20)
    dig = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    nwg = (n + 63) // 64
    for mode in modes:
        lib.cg_diag_sha_mode(mode)
        st = torch.cuda.current_stream().cuda_stream
        args = (data.data_ptr(), offs_t.data_ptr(), lens_t.data_ptr(), n, 1, dig.data_ptr(), st)
        assert lib.cg_hash_spans_device(*args) == 0
        torch.cuda.synchronize()
        lib.cg_diag_sha_stats(nwg, None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.cg_hash_spans_device(*args) == 0
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros(4 * nwg, np.uint64)
        lib.cg_diag_sha_stats(nwg, buf.ctypes.data)
        lib.cg_diag_sha_stats(0, None)
        b = buf.reshape(-1, 4).astype(float)
        rounds = (BIG // 64 + 1) * 64
        res[f"{name}/mode{mode}"] = {"ms": e0.elapsed_time(e1),
                                     "cyc_per_round_max": float(b[:, 3].max() / rounds),
                                     "cyc_per_round_min": float(b[:, 3][b[:, 3] > 0].min() / rounds),
                                     "prod_spin_frac_med": float(np.median(b[:, 0] / np.maximum(b[:, 1], 1)))}
        print(name, mode, res[f"{name}/mode{mode}"], file=sys.stderr, flush=True)
lib.cg_diag_sha_mode(0)
print(json.dumps(res, indent=1))
