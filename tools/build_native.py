#!/usr/bin/env python3
"""Build the mp4x native libraries in-tree (gfx950).

* ``mp4x/_native/libmp4x_hip.so``  — HIP kernels (csrc/kernels/*.hip) + device runtime
  (csrc/runtime/*.hip): compiled with ``hipcc --offload-arch=gfx950`` and linked against the
  SAME ``libamdhip64.so`` that PyTorch-ROCm loads (torch/lib), so kernels launch on torch's
  streams inside one HIP runtime instance.
* ``mp4x/_native/libmp4x_host.so`` — host runtime (csrc/host/*.cpp): CPU reduction kernels,
  the TCP data-plane engine; plain g++, no GPU dependency.
* ``mp4x/_native/_mp4x_team*.so`` — CPython extension (csrc/pyext/team_ext.cpp) binding the
  host runtime's thread team for ThreadCommSlave (buffer protocol + one FASTCALL per phase),
  linked against libmp4x_host.so next to it (rpath $ORIGIN).
* ``mp4x/_native/_mp4x_map*.so`` — CPython extension over libtorch (csrc/pyext/map_ext.cpp): the
  device map collectives' Dict[key, Tensor] -> ids / rows walk.
* ``mp4x/_native/_mp4x_hostmap*.so`` — CPython + numpy C-API extension (csrc/pyext/hostmap_ext.cpp):
  the host map collectives' Java-hash owner partition and value-row stacking.

Incremental: objects are rebuilt only when a source or header is newer.
``--debug`` builds ``libmp4x_hip_debug.so`` instead: ``-O1 -g -DMP4X_DEBUG``, which turns on the
device-side bounds asserts (``MP4X_DASSERT``: printf + trap) in the kernels; load it with
``MP4X_NATIVE_DEBUG=1`` (SURVEY §5.2 "HIP kernel bounds checks in debug builds").
Usage: python tools/build_native.py [--clean] [--debug] [-j N]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "mp4x", "_native")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("MP4X_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")).split(";")[0]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def torch_lib_dir():
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.exists(os.path.join(d, "libamdhip64.so")):
                return d
    except Exception:
        pass
    return None


def headers():
    return [f for ext in ("*.h", "*.hpp") for f in glob.glob(os.path.join(CSRC, "**", ext), recursive=True)]


def newer(src, obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in deps)


def run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise SystemExit(f"build failed: {cmd[-1]}")
    return r.stdout


def build_hip(jobs, debug=False):
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "runtime", "*.hip")))
    deps = headers()
    objdir = OBJ + ("_debug" if debug else "")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if newer(s, o, deps):
            todo.append((s, o))

    def comp(so):
        s, o = so
        opt = ["-O1", "-g", "-DMP4X_DEBUG"] if debug else ["-O3"]
        # the IPC kernels' register / LDS budgets are kept next to the library: the shared-GPU
        # co-residency caps are derived from them (mp4x/parallel/occupancy.py)
        res = not debug and os.path.basename(s).startswith("ipc")
        out = run([HIPCC, f"--offload-arch={ARCH}"] + opt + ["-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result"]
                  + (["-Rpass-analysis=kernel-resource-usage"] if res else [])
                  + ["-I", os.path.join(CSRC, "include"), "-c", s, "-o", o])
        if res:
            with open(o + ".res.txt", "w") as f:
                f.write(out)
        return s

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in ex.map(comp, todo):
            print("  hipcc", os.path.relpath(s, ROOT))
    out = os.path.join(OUT, "libmp4x_hip_debug.so" if debug else "libmp4x_hip.so")
    if not debug:
        table = os.path.join(OUT, "ipc_kernel_resources.json")
        if todo or not os.path.exists(table):
            write_resource_table(sorted(o for o in objs if os.path.basename(o).startswith("ipc")), table)
    if todo or not os.path.exists(out):
        tl = torch_lib_dir()
        libdir = tl or "/opt/rocm/lib"
        # Link with the host compiler (not hipcc, which would add /opt/rocm's libamdhip64.so.7):
        # the kernels must bind to the SAME HIP runtime instance PyTorch-ROCm loaded, or torch's
        # stream handles and device pointers would belong to a different runtime.
        link = ["g++", "-shared", "-fPIC", "-o", out] + objs
        if tl:
            link += ["-L", tl, "-l:libamdhip64.so", "-Wl,-rpath," + tl]
        else:
            link += ["-L", libdir, "-lamdhip64", "-Wl,-rpath," + libdir]
        run(link)
        print("  link ", os.path.relpath(out, ROOT), "(hip runtime from", libdir + ")")
    return out


def parse_resource_remarks(text):
    """{mangled kernel name: {"sgpr", "vgpr", "agpr", "lds", "occ"}} from the compiler's
    ``-Rpass-analysis=kernel-resource-usage`` remarks."""
    import re
    keys = {"TotalSGPRs": "sgpr", "VGPRs": "vgpr", "AGPRs": "agpr", "LDS Size [bytes/block]": "lds",
            "Occupancy [waves/SIMD]": "occ"}
    table, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = table.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z][^:]*?): (\d+) \[", line)
        if m and cur is not None and m.group(1) in keys:
            cur[keys[m.group(1)]] = int(m.group(2))
    return table


def write_resource_table(objs, path):
    """Demangled IPC kernel name -> resources, from the remarks saved at compile time."""
    import json
    table = {}
    for o in objs:
        try:
            with open(o + ".res.txt") as f:
                table.update(parse_resource_remarks(f.read()))
        except OSError:
            pass
    names = list(table)
    dem = names
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), stdout=subprocess.PIPE, text=True, check=True)
        dem = r.stdout.split("\n")[:len(names)]
    except Exception:   # noqa: BLE001 — mangled names still parse for the family prefix
        pass
    out = {d: table[n] for n, d in zip(names, dem) if "k_ipc" in d}
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("  wrote", os.path.relpath(path, ROOT), f"({len(out)} kernels)")


def build_host(jobs):
    srcs = sorted(f for f in glob.glob(os.path.join(CSRC, "host", "*.cpp"))
                  if not os.path.basename(f).startswith("test_"))   # test_*.cpp are standalone test programs
    if not srcs:
        return None
    deps = headers()
    os.makedirs(OBJ, exist_ok=True)
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if newer(s, o, deps):
            todo.append((s, o))

    def comp(so):
        s, o = so
        run(["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-fPIC", "-Wall", "-pthread",
             "-I", os.path.join(CSRC, "include"), "-c", s, "-o", o])
        return s

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in ex.map(comp, todo):
            print("  g++  ", os.path.relpath(s, ROOT))
    out = os.path.join(OUT, "libmp4x_host.so")
    if todo or not os.path.exists(out):
        run(["g++", "-shared", "-fPIC", "-pthread", "-o", out] + objs)
        print("  link ", os.path.relpath(out, ROOT))
    return out


def build_pyext(host_so):
    import sysconfig
    src = os.path.join(CSRC, "pyext", "team_ext.cpp")
    if not host_so or not os.path.exists(src):
        return None
    out = os.path.join(OUT, "_mp4x_team" + sysconfig.get_config_var("EXT_SUFFIX"))
    if newer(src, out, headers()) or os.path.getmtime(host_so) > os.path.getmtime(out):
        run(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-shared", "-I", sysconfig.get_paths()["include"],
             src, "-o", out, "-L", OUT, "-l:libmp4x_host.so", "-Wl,-rpath,$ORIGIN"])
        print("  g++  ", os.path.relpath(src, ROOT), "->", os.path.relpath(out, ROOT))
    return out


def build_hostmapext():
    """``_mp4x_hostmap``: plain CPython extension (no torch) for the host map collectives."""
    import sysconfig
    src = os.path.join(CSRC, "pyext", "hostmap_ext.cpp")
    out = os.path.join(OUT, "_mp4x_hostmap" + sysconfig.get_config_var("EXT_SUFFIX"))
    if os.path.exists(src) and newer(src, out, []):
        import numpy
        run(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-shared", "-I", sysconfig.get_paths()["include"],
             "-I", numpy.get_include(), src, "-o", out])
        print("  g++  ", os.path.relpath(src, ROOT), "->", os.path.relpath(out, ROOT))
    return out


def build_launchext():
    """``_mp4x_launch``: plain CPython extension, the ctypes-free per-call launch of the IPC
    allreduce (csrc/pyext/launch_ext.cpp; calls libmp4x_hip.so through a bound pointer)."""
    import sysconfig
    src = os.path.join(CSRC, "pyext", "launch_ext.cpp")
    out = os.path.join(OUT, "_mp4x_launch" + sysconfig.get_config_var("EXT_SUFFIX"))
    if os.path.exists(src) and newer(src, out, []):
        run(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-shared", "-I", sysconfig.get_paths()["include"],
             src, "-o", out])
        print("  g++  ", os.path.relpath(src, ROOT), "->", os.path.relpath(out, ROOT))
    return out


def build_mapext():
    """``_mp4x_map``: CPython extension reading ``at::Tensor`` facts directly (libtorch headers,
    linked against the torch libraries PyTorch itself loads; rpath to torch/lib)."""
    import sysconfig
    src = os.path.join(CSRC, "pyext", "map_ext.cpp")
    tl = torch_lib_dir()
    if not os.path.exists(src) or tl is None:
        return None
    import torch
    tinc = os.path.join(os.path.dirname(tl), "include")
    out = os.path.join(OUT, "_mp4x_map" + sysconfig.get_config_var("EXT_SUFFIX"))
    if newer(src, out, []):
        abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
        run(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-I", sysconfig.get_paths()["include"], "-isystem", tinc,
             "-isystem", os.path.join(tinc, "torch", "csrc", "api", "include"),
             src, "-o", out, "-L", tl, "-ltorch_python", "-ltorch", "-ltorch_cpu", "-lc10", "-Wl,-rpath," + tl])
        print("  g++  ", os.path.relpath(src, ROOT), "->", os.path.relpath(out, ROOT))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true", help="device-assert build -> libmp4x_hip_debug.so")
    a = ap.parse_args(argv)
    if a.clean:
        shutil.rmtree(os.path.join(ROOT, "build"), ignore_errors=True)
        for f in glob.glob(os.path.join(OUT, "*.so")):
            os.remove(f)
    os.makedirs(OUT, exist_ok=True)
    print(f"mp4x native build (arch {ARCH}{', debug' if a.debug else ''})")
    if a.debug:
        build_hip(a.j, debug=True)
        return 0
    build_hip(a.j)
    build_pyext(build_host(a.j))
    build_mapext()
    build_hostmapext()
    build_launchext()
    return 0


if __name__ == "__main__":
    sys.exit(main())
