"""Diagnostic: device memory visible to one process -- hipMemGetInfo, then
hipMalloc of CHUNK-GB blocks until one fails (all freed at the end).
Usage: python profiles/diag/mem_probe.py [CHUNK_GB]"""
import ctypes as C
import sys

hip = C.CDLL("libamdhip64.so")
chunk = int(float(sys.argv[1] if len(sys.argv) > 1 else 16) * (1 << 30))
free, tot = C.c_size_t(), C.c_size_t()
hip.hipMemGetInfo(C.byref(free), C.byref(tot))
print(f"total {tot.value / 2**30:.1f} GiB, free {free.value / 2**30:.1f} GiB", flush=True)
ptrs = []
while True:
    p = C.c_void_p()
    rc = hip.hipMalloc(C.byref(p), C.c_size_t(chunk))
    if rc != 0:
        break
    ptrs.append(p)
hip.hipMemGetInfo(C.byref(free), C.byref(tot))
print(f"allocated {len(ptrs)} x {chunk / 2**30:.1f} GiB = {len(ptrs) * chunk / 2**30:.1f} GiB; "
      f"free now {free.value / 2**30:.1f} GiB", flush=True)
for p in ptrs:
    hip.hipFree(p)
