"""Native build driver: compiles csrc/ into in-tree shared libraries.

* ``libstereo_amd.so``  — HIP kernels (gfx950) + engine runtime + models + C API (hipcc)
* ``libstereo_host.so`` — CPU-only geometry / calibration / image I/O (g++), loadable without a GPU

Incremental (object timestamps vs. sources and headers), parallel.  Used by
``__graft_entry__.build()`` and ``python -m stereoalgorithms_amd._build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "lib"
OBJDIR = ROOT / "build" / "obj"
ARCH = os.environ.get("SA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX_HOST", "g++")

HOST_DIRS = ("host",)  # CPU-only sources -> libstereo_host.so
DEVICE_DIRS = ("kernels", "runtime", "models", "api")

BINDIR = Path(__file__).resolve().parent / "bin"
# csrc/abi source -> library exporting the reference's symbol names
ABI_LIBS = {"raftstereo_abi.cpp": "libRAFTStereo.so", "hitnet_abi.cpp": "libHitNet.so",
            "crestereo_abi.cpp": "libCREStereo.so", "fastacvnet_abi.cpp": "libFastACVNet_plus.so"}
# apps source -> ABI library it links (reference demo executable names)
APPS = {"raft_stereo_demo.cpp": "libRAFTStereo.so", "HitNet_demo.cpp": "libHitNet.so",
        "crestereo_demo.cpp": "libCREStereo.so", "fastacvnet_plus_demo.cpp": "libFastACVNet_plus.so",
        "Stereo_Calibration.cpp": "libstereo_host.so", "stereo_capture.cpp": "libstereo_host.so",
        "abi_check.cpp": "libstereo_host.so"}

COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", "-Wall", "-Wno-unused-function"]


def _headers_mtime() -> float:
    hs = list((CSRC / "include").rglob("*.h")) + list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _sources(dirs):
    out = []
    for d in dirs:
        out += sorted((CSRC / d).rglob("*.hip")) + sorted((CSRC / d).rglob("*.cpp"))
    return out


def _compile(src: Path, obj: Path, host_only: bool, hmt: float, verbose: bool) -> str | None:
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hmt):
        return None
    obj.parent.mkdir(parents=True, exist_ok=True)
    if host_only:
        cmd = [CXX, *COMMON_FLAGS, f"-I{CSRC / 'abi'}", "-c", str(src), "-o", str(obj)]
    else:
        cmd = [HIPCC, f"--offload-arch={ARCH}", *COMMON_FLAGS, "-c", str(src), "-o", str(obj)]
        if src.suffix == ".hip":
            cmd[1:1] = ["-x", "hip"]
        cmd += [f"-I{CSRC / 'models'}", "-munsafe-fp-atomics"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return str(src.relative_to(ROOT))


def _link(objs, out: Path, host_only: bool, extra=(), shared: bool = True):
    newest = max(o.stat().st_mtime for o in objs)
    # the object set is part of the link's inputs: a deleted / added source relinks too
    manifest = OBJDIR / "link" / (out.name + ".objs")
    objset = "\n".join(sorted(map(str, objs))) + "\n" + " ".join(extra)
    same = manifest.exists() and manifest.read_text() == objset
    if same and out.exists() and out.stat().st_mtime >= newest:
        return False
    out.parent.mkdir(parents=True, exist_ok=True)
    if host_only:
        cmd = [CXX, *(["-shared"] if shared else []), "-o", str(out), *map(str, objs), *extra]
    else:
        cmd = [HIPCC, f"--offload-arch={ARCH}", *(["-shared"] if shared else []), "-o", str(out),
               *map(str, objs), *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{r.stdout}\n{r.stderr}")
    manifest.parent.mkdir(parents=True, exist_ok=True)
    manifest.write_text(objset)
    return True


def build(jobs: int | None = None, verbose: bool = False) -> dict:
    jobs = jobs or min(16, os.cpu_count() or 4)
    hmt = _headers_mtime()
    host_src = _sources(HOST_DIRS)
    dev_src = _sources(DEVICE_DIRS)
    tasks = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in host_src:
            tasks.append(ex.submit(_compile, s, OBJDIR / "host" / (s.stem + s.suffix + ".o"), True, hmt, verbose))
        for s in dev_src:
            tasks.append(ex.submit(_compile, s, OBJDIR / "dev" / (s.stem + s.suffix + ".o"), False, hmt, verbose))
        built = [t.result() for t in tasks]
    built = [b for b in built if b]
    host_lib = LIBDIR / "libstereo_host.so"
    dev_lib = LIBDIR / "libstereo_amd.so"
    host_objs = [OBJDIR / "host" / (s.stem + s.suffix + ".o") for s in host_src]
    dev_objs = [OBJDIR / "dev" / (s.stem + s.suffix + ".o") for s in dev_src]
    if host_objs:
        _link(host_objs, host_lib, True, extra=["-lz"])
    roctx = ["-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
    _link(dev_objs, dev_lib, False,
          extra=([f"-L{LIBDIR}", "-lstereo_host", "-Wl,-rpath,$ORIGIN"] if host_objs else []) + roctx)
    libs = [str(host_lib), str(dev_lib)]
    # reference-compatible per-model C ABI libraries + demo executables (host compiler, link the
    # engine library)
    abi_built = []
    for src, lib in ABI_LIBS.items():
        s = CSRC / "abi" / src
        obj = OBJDIR / "abi" / (s.stem + ".o")
        r = _compile(s, obj, True, hmt, verbose)
        if r:
            abi_built.append(r)
        out = LIBDIR / lib
        _link([obj], out, True, extra=[f"-L{LIBDIR}", "-lstereo_amd", "-lstereo_host", "-Wl,-rpath,$ORIGIN"])
        libs.append(str(out))
    BINDIR.mkdir(parents=True, exist_ok=True)
    for app, lib in APPS.items():
        s = ROOT / "apps" / app
        obj = OBJDIR / "apps" / (s.stem + ".o")
        r = _compile(s, obj, True, max(hmt, (ROOT / "apps" / "demo_main.h").stat().st_mtime), verbose)
        if r:
            abi_built.append(r)
        libname = lib[3:-3]
        _link([obj], BINDIR / s.stem, True, shared=False,
              extra=[f"-L{LIBDIR}", f"-l{libname}", "-lstereo_host", "-ldl", "-Wl,-rpath,$ORIGIN/../lib"])
    # native RCCL data parallelism: its own library (Python processes never load a second RCCL next to
    # torch's) + the C++ multi-GPU bench
    dsrc = CSRC / "dist" / "dist.cpp"
    dobj = OBJDIR / "dist" / "dist.cpp.o"
    r = _compile(dsrc, dobj, False, hmt, verbose)
    if r:
        abi_built.append(r)
    dist_lib = LIBDIR / "libstereo_dist.so"
    _link([dobj], dist_lib, False, extra=[f"-L{LIBDIR}", "-lstereo_amd", "-L/opt/rocm/lib", "-lrccl",
                                          "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])
    libs.append(str(dist_lib))
    s = ROOT / "apps" / "stereo_bench_dp.cpp"
    obj = OBJDIR / "apps" / "stereo_bench_dp.o"
    r = _compile(s, obj, False, hmt, verbose)
    if r:
        abi_built.append(r)
    _link([obj], BINDIR / "stereo_bench_dp", False, shared=False,
          extra=[f"-L{LIBDIR}", "-lstereo_dist", "-lstereo_amd", "-lstereo_host", "-Wl,-rpath,$ORIGIN/../lib"])
    # standalone HIP diagnostics (tools/graph_repro: graph-replay stability without the engine)
    gdir = ROOT / "tools" / "graph_repro"
    for src, out, extra in (("graph_capture_repro.hip", "graph_capture_repro", []),
                            ("overlap_repro.hip", "overlap_repro", []),
                            ("xq_latency.hip", "xq_latency", []),
                            ("other_kernel.hip", "other_kernel.hsaco", ["--genco"])):
        s, o = gdir / src, BINDIR / out
        if not o.exists() or o.stat().st_mtime < s.stat().st_mtime:
            r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-O2", *extra, "-o", str(o), str(s)],
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {s}\n{r.stderr}")
            abi_built.append(str(s.relative_to(ROOT)))
    return {"compiled": built + abi_built, "libs": libs}


if __name__ == "__main__":
    info = build(verbose="-v" in sys.argv)
    print(f"compiled {len(info['compiled'])} files -> {info['libs']}")
