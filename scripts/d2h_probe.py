"""Diagnostic: host-observed latency of small device->pinned-host copies (hipMemcpyAsync + hipStreamSynchronize)
for the result sizes the evaluator returns (C2: 240 rows, C4: 24000 rows), per hipHostMalloc flag."""
import ctypes, time
hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
def ok(e):
    assert e == 0, e
dev = vp(); ok(hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(64 << 20)))
st = vp(); ok(hip.hipStreamCreate(ctypes.byref(st)))
for flags, fname in ((0, "Default"), (0x4, "Coherent"), (0x8, "NonCoherent")):
    host = vp(); ok(hip.hipHostMalloc(ctypes.byref(host), ctypes.c_size_t(16 << 20), ctypes.c_uint(flags)))
    for rows in (240, 24000, 240000):
        for ncopy in (1, 4):
            ts = []
            for it in range(20):
                t = time.perf_counter()
                per = rows * 8
                for c in range(ncopy):
                    ok(hip.hipMemcpyAsync(vp(host.value + c * per), vp(dev.value + c * per), ctypes.c_size_t(per), 2, st))
                ok(hip.hipStreamSynchronize(st))
                ts.append(time.perf_counter() - t)
            ts = sorted(ts)[2:-2]
            print(f"{fname:12s} rows={rows:7d} copies={ncopy}: {1e3 * sum(ts) / len(ts):.3f} ms", flush=True)
    ok(hip.hipHostFree(host))
