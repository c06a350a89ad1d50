"""Diagnostic: how long hipMalloc / hipFree of a stream arena take (the stream handle grows
its arena to the whole in-flight budget in one allocation).  Sizes in MiB; each
allocation is timed cold and after a free of the same size.  Prints one JSON object."""
import ctypes
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402,F401  (loads the HIP runtime the package uses)

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipDeviceSynchronize.argtypes = []
res = {}
hip.hipDeviceSynchronize()
for mib in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "256,1024,2048,3072,4096,6144,8192").split(",")]:
    row = []
    for _ in range(2):
        p = ctypes.c_void_p()
        t0 = time.perf_counter()
        assert hip.hipMalloc(ctypes.byref(p), mib << 20) == 0
        t1 = time.perf_counter()
        assert hip.hipFree(p) == 0
        t2 = time.perf_counter()
        row.append({"malloc_ms": round((t1 - t0) * 1e3, 3), "free_ms": round((t2 - t1) * 1e3, 3)})
    res[f"{mib}MiB"] = row
print(json.dumps(res))
