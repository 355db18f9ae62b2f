#!/usr/bin/env python3
"""In-tree native build for dtg (no setuptools, no hipify, no JIT cache).

Produces two extension modules inside the package directory:

* ``_C``        -- hand-written gfx950 HIP kernels + their PyTorch bindings (hipcc, torch headers)
* ``_runtime``  -- the C++ runtime: parameter-server service, accumulator/token queue,
                   TensorBundle checkpoint I/O (g++, pybind11, no GPU dependency)

Objects are cached under ``build/obj`` keyed by a hash of (source, headers, flags), so a rebuild
after editing one kernel only recompiles that file.  Usage::

    python tools/build_ext.py [--only C|runtime] [-j N] [--verbose]
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-tensorflow-guide_amd")
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("DTG_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _torch_paths():
    import torch  # noqa: local import keeps `--only runtime` torch-free
    base = os.path.dirname(torch.__file__)
    return (os.path.join(base, "include"), os.path.join(base, "include", "torch", "csrc", "api", "include"),
            os.path.join(base, "lib"), bool(torch._C._GLIBCXX_USE_CXX11_ABI))


def _pybind_include():
    import pybind11
    return pybind11.get_include()


_INC = re.compile(rb'^\s*#\s*include\s*"([^"]+)"', re.M)


def _headers_digest(src=None):
    """Digest of the project headers a source includes (transitively, quoted includes resolved against
    csrc/include and the including file's directory); without a source, of every project header."""
    h = hashlib.sha256()
    if src is None:
        for p in sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) +
                        glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)):
            with open(p, "rb") as f:
                h.update(p.encode())
                h.update(f.read())
        return h.hexdigest()
    seen, todo = set(), [src]
    while todo:
        cur = todo.pop()
        with open(cur, "rb") as f:
            body = f.read()
        for inc in _INC.findall(body):
            inc = inc.decode()
            for base in (os.path.join(CSRC, "include"), os.path.dirname(cur)):
                cand = os.path.normpath(os.path.join(base, inc))
                if os.path.exists(cand):
                    if cand not in seen:
                        seen.add(cand)
                        todo.append(cand)
                    break
    for p in sorted(seen):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


def _compile(src, cmd_prefix, flags, hdr_digest, verbose):
    with open(src, "rb") as f:
        body = f.read()
    hdr_digest = _headers_digest(src)  # only the headers this source actually includes
    key = hashlib.sha256(body + hdr_digest.encode() + " ".join(cmd_prefix + flags).encode()).hexdigest()[:20]
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(OBJ, f"{rel}.{key}.o")
    if os.path.exists(obj):
        return obj, False
    cmd = cmd_prefix + flags + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip() and verbose:
        print(r.stderr)
    os.replace(obj + ".tmp", obj)
    return obj, True


def _link(objs, out, cmd):
    tmp = out + ".tmp"
    r = subprocess.run(cmd + objs + ["-o", tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


def build_C(jobs=8, verbose=False, name="_C", kdir="kernels", bdir="bindings"):
    """A torch extension from csrc/<kdir>/*.hip (hipcc, gfx950) and csrc/<bdir>/*.cc: the production kernels
    (_C), or the A/B lab kernels (_lab: csrc/lab, tools only -- never imported by the package)."""
    tinc, tapi, tlib, cxx11 = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{os.path.join(CSRC, 'include')}",
              f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}"]
    hip_flags = common + [f"--offload-arch={ARCH}", "-ffp-contract=fast", "-Wno-unused-result",
                          "-munsafe-fp-atomics"]
    bind_flags = common + [f"-I{os.path.join(ROCM, 'include')}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
                           f"-DTORCH_EXTENSION_NAME={name}", f"-I{tinc}", f"-I{tapi}", f"-I{pyinc}",
                           "-Wno-unused-parameter", "-Wno-deprecated-declarations"]
    kern = sorted(glob.glob(os.path.join(CSRC, kdir, "*.hip")))
    binds = sorted(glob.glob(os.path.join(CSRC, bdir, "*.cc")))
    hd = _headers_digest()
    os.makedirs(OBJ, exist_ok=True)
    objs, built = [], 0
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, [HIPCC], hip_flags, hd, verbose) for s in kern]
        futs += [ex.submit(_compile, s, ["g++"], bind_flags, hd, verbose) for s in binds]
        for f in futs:
            o, b = f.result()
            objs.append(o)
            built += b
    out = os.path.join(PKG, name + EXT)
    if built or not os.path.exists(out):
        _link(objs, out, [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", f"-L{tlib}",
                          "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                          f"-Wl,-rpath,{tlib}"])
    return out


def build_runtime(jobs=8, verbose=False):
    pyinc = sysconfig.get_paths()["include"]
    flags = ["-O2", "-g", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-parameter",
             f"-I{os.path.join(CSRC, 'include')}", f"-I{_pybind_include()}", f"-I{pyinc}",
             "-fvisibility=hidden"]
    extra = os.environ.get("DTG_RUNTIME_CXXFLAGS", "").split()
    flags += extra
    srcs = sorted(glob.glob(os.path.join(CSRC, "ps", "*.cc")) + glob.glob(os.path.join(CSRC, "ckpt", "*.cc")) +
                  glob.glob(os.path.join(CSRC, "runtime", "*.cc")))
    hd = _headers_digest()
    os.makedirs(OBJ, exist_ok=True)
    objs, built = [], 0
    with cf.ThreadPoolExecutor(jobs) as ex:
        for o, b in ex.map(lambda s: _compile(s, ["g++"], flags, hd, verbose), srcs):
            objs.append(o)
            built += b
    out = os.path.join(PKG, "_runtime" + EXT)
    if built or not os.path.exists(out):
        _link(objs, out, ["g++", "-shared", "-fPIC", "-pthread"] + extra)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["C", "runtime", "lab"], default=None)
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args(argv)
    if a.clean and os.path.isdir(OBJ):
        shutil.rmtree(OBJ)
    if a.only in (None, "runtime"):
        print("built", build_runtime(a.j, a.verbose))
    if a.only in (None, "C"):
        print("built", build_C(a.j, a.verbose))
    if a.only == "lab":  # the A/B lab extension: only on request (tools), never part of the package build
        print("built", build_C(a.j, a.verbose, name="_lab", kdir="lab", bdir="lab"))


if __name__ == "__main__":
    sys.exit(main())
