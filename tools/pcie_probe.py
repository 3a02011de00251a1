"""Host->device copy rates on the GPU box, for the PCIe-inclusive wakeup
(DESIGN §5): one C2 wakeup batch is ~43 MB.  hipMemcpy of the same bytes from
(a) pageable numpy memory, (b) the same memory registered with hipHostRegister
(what crgc_host_register does), (c) hipHostMalloc memory; each as one copy and
as 44 copies of ~1 MB (the chunked merge's pattern: 4 chunks x 11 arrays).

usage: python tools/pcie_probe.py [MB]
"""
import ctypes as C
import sys
import time

import numpy as np

hip = C.CDLL("libamdhip64.so")
H2D = 1


def ok(e, what):
    if e != 0:
        raise RuntimeError(f"{what}: hip error {e}")


def timed(fn, reps=5):
    fn()
    ok(hip.hipDeviceSynchronize(), "sync")
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    ok(hip.hipDeviceSynchronize(), "sync")
    return (time.perf_counter() - t) / reps


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 43
    n = mb << 20
    dev = C.c_void_p()
    ok(hip.hipMalloc(C.byref(dev), C.c_size_t(n)), "hipMalloc")
    page = np.ones(n, dtype=np.uint8)
    reg = np.ones(n + 4096, dtype=np.uint8)
    off = (-reg.ctypes.data) % 4096
    regp = reg.ctypes.data + off
    ok(hip.hipHostRegister(C.c_void_p(regp), C.c_size_t(n), 0), "hipHostRegister")
    hm = C.c_void_p()
    ok(hip.hipHostMalloc(C.byref(hm), C.c_size_t(n), 0), "hipHostMalloc")
    C.memset(hm, 1, n)
    stream = C.c_void_p()
    ok(hip.hipStreamCreate(C.byref(stream)), "stream")

    def one(src):
        return lambda: ok(hip.hipMemcpyAsync(dev, C.c_void_p(src), C.c_size_t(n), H2D, stream), "copy")

    def many(src, k=44):
        step = n // k

        def f():
            for i in range(k):
                ok(hip.hipMemcpyAsync(C.c_void_p(dev.value + i * step), C.c_void_p(src + i * step),
                                      C.c_size_t(step), H2D, stream), "copy")
        return f

    out = {}
    for name, src in (("pageable", page.ctypes.data), ("registered", regp), ("hostmalloc", hm.value)):
        t1 = timed(one(src))
        t2 = timed(many(src))
        out[name] = {"one_copy_ms": t1 * 1e3, "one_copy_GBs": n / t1 / 1e9,
                     "44_copies_ms": t2 * 1e3, "44_copies_GBs": n / t2 / 1e9}
        print(name, {k: round(v, 3) for k, v in out[name].items()}, flush=True)
    hip.hipHostUnregister(C.c_void_p(regp))
    hip.hipHostFree(hm)
    hip.hipFree(dev)


if __name__ == "__main__":
    main()
