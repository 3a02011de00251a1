"""Build the HIP shim in-tree: uigc-akka_amd/lib/libcrgc_hip.so (gfx950 only)."""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "lib")
SOURCES = ["crgc_api.hip", "crgc_merge.hip", "crgc_trace.hip", "crgc_rebuild.hip",
           "crgc_transport.hip", "crgc_route.hip", "crgc_delta.hip",
           "crgc_undo.hip", "crgc_chain.hip", "crgc_edges.hip", "crgc_xchain.hip", "crgc_reuse.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
         "-Wno-unused-function", "-Wno-unused-result", "-Wno-unused-value", "-munsafe-fp-atomics"]


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(os.path.join(OUT, "obj"), exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")]
    headers.append(os.path.join(os.path.dirname(PKG), "include", "crgc.h"))
    lib = os.path.join(OUT, "libcrgc_hip.so")
    jobs = []
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(OUT, "obj", src.replace(".hip", ".o"))
        objs.append(o)
        if force or _stale(o, [s] + headers):
            jobs.append([HIPCC, *FLAGS, "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        for cmd, r in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
            if verbose or r.returncode:
                print(" ".join(cmd)); print(r.stdout, r.stderr)
            if r.returncode:
                raise RuntimeError(f"hipcc failed: {cmd[-3]}")
    if force or jobs or _stale(lib, objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            print(r.stdout, r.stderr)
            raise RuntimeError("link failed")
    return lib


if __name__ == "__main__":
    print(build(verbose=True))
