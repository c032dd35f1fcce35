"""D->H copy rates of the 7.68 MB framebuffer (800x800 float3) into pageable, hipHostRegister'ed
and hipHostMalloc'ed host memory, with hipMemcpy and hipMemcpyAsync + stream sync (the pt_trace
copy, pathtrace.cu:783).  Prints one JSON line.  Tools only."""
import ctypes
import json
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
hip.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
hip.hipStreamSynchronize.argtypes = [vp]
D2H = 2
N = 800 * 800 * 12


def timed(fn, reps=30):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(1e3 * ts[len(ts) // 2], 4)


def main():
    d = vp()
    assert hip.hipMalloc(ctypes.byref(d), N) == 0
    st = vp()
    assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    out = {}
    page = np.empty(N, np.uint8)
    out["pageable_memcpy_ms"] = timed(lambda: hip.hipMemcpy(page.ctypes.data, d, N, D2H))
    reg = np.empty(N + 4096, np.uint8)
    rc = hip.hipHostRegister(reg.ctypes.data, N, 0)
    out["register_rc"] = rc
    out["registered_memcpy_ms"] = timed(lambda: hip.hipMemcpy(reg.ctypes.data, d, N, D2H))

    def asy(p):
        hip.hipMemcpyAsync(p, d, N, D2H, st)
        hip.hipStreamSynchronize(st)
    out["registered_async_ms"] = timed(lambda: asy(reg.ctypes.data))
    out["pageable_async_ms"] = timed(lambda: asy(page.ctypes.data))
    h = vp()
    assert hip.hipHostMalloc(ctypes.byref(h), N, 0) == 0
    out["hostmalloc_memcpy_ms"] = timed(lambda: hip.hipMemcpy(h, d, N, D2H))
    out["hostmalloc_async_ms"] = timed(lambda: asy(h))
    host = np.empty(N, np.uint8)
    out["host_memcpy_7_68MB_ms"] = timed(lambda: ctypes.memmove(host.ctypes.data, h, N))
    out["GBps_best"] = round(N / 1e6 / min(v for k, v in out.items() if k.endswith("_ms")), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
