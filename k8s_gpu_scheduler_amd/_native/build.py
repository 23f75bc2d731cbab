"""Build the native extension modules in-tree (gfx950 only).

  _core  native/core/*.cpp   host C++ (g++)            scoring core
  _smi   native/smi/*.cpp    host C++ + libamd_smi     telemetry / topology / partitions
  _hip   native/hip/*        hipcc --offload-arch=gfx950  device query, CU-masked streams,
                                                        MFMA/HBM load kernels, xGMI probes

`python -m k8s_gpu_scheduler_amd._native.build [--force] [--asan]` (also called by
`__graft_entry__.build()`).  Outputs land next to this file so they travel with the repo
snapshot to the GPU box.  `--asan` builds the host-only modules with
-fsanitize=address,undefined (host sanitizers only; GPU ASan is not used).
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import List, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
NATIVE = os.path.join(REPO, "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"],
              "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"]}


def _targets(asan: bool = False, san_kind: str = "") -> List[Tuple[str, List[str], List[str]]]:
    inc = _py_includes()
    san = SANITIZERS.get(san_kind or ("asan" if asan else ""), [])
    core_src = sorted(glob.glob(os.path.join(NATIVE, "core", "*.cpp")))
    smi_src = sorted(glob.glob(os.path.join(NATIVE, "smi", "*.cpp")))
    hip_src = sorted(glob.glob(os.path.join(NATIVE, "hip", "*.hip")) + glob.glob(os.path.join(NATIVE, "hip", "*.cpp")))
    out = [
        ("_core", core_src, ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", *san, *inc, *core_src]),
        ("_smi", smi_src, ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", *san, *inc, f"-I{ROCM}/include",
                           *smi_src, f"-L{ROCM}/lib", "-lamd_smi", f"-Wl,-rpath,{ROCM}/lib", "-pthread"]),
        ("_hip", hip_src, [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17",
                           "-shared", "-fPIC", *inc, *hip_src, f"-Wl,-rpath,{ROCM}/lib"]),
    ]
    return out


def _stale(out: str, srcs: List[str]) -> bool:
    if not os.path.exists(out):
        return True
    deps = srcs + glob.glob(os.path.join(NATIVE, "**", "*.h"), recursive=True)
    mt = os.path.getmtime(out)
    return any(os.path.getmtime(s) > mt for s in deps)


def build(force: bool = False, asan: bool = False, only: Tuple[str, ...] = (), verbose: bool = False,
          san_kind: str = "") -> List[str]:
    """san_kind: "" | "asan" (address+undefined) | "tsan" (thread) -- host modules only."""
    built = []
    jobs = []
    kind = san_kind or ("asan" if asan else "")
    for name, srcs, cmd in _targets(asan, kind):
        if only and name not in only:
            continue
        if kind and name == "_hip":
            continue                # GPU code is never built with a host sanitizer
        out = os.path.join(HERE, name + (f"_{kind}" if kind else "") + EXT)
        if not force and not _stale(out, srcs):
            continue
        jobs.append((name, out, cmd + ["-o", out + ".tmp"]))

    def run(job):
        name, out, cmd = job
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"building {name} failed:\n{p.stderr[-4000:]}")
        os.replace(out + ".tmp", out)
        return out

    with ThreadPoolExecutor(max(1, len(jobs))) as ex:
        built = list(ex.map(run, jobs))
    if not kind and (not only or "cy" in only):
        # the compiled control-plane modules (Cython; skipped when Cython is absent)
        from . import cyaccel
        built += cyaccel.build(force=force, verbose=verbose)
    return built


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true")
    ap.add_argument("--tsan", action="store_true")
    ap.add_argument("--only", nargs="*", default=[])
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    for p in build(a.force, a.asan, tuple(a.only), a.verbose, "tsan" if a.tsan else ""):
        print("built", p)


def sampler_tsan_test(workdir: str) -> Tuple[int, str]:
    """Build and run native/tests/sampler_tsan.cpp under ThreadSanitizer (host)."""
    exe = os.path.join(workdir, "sampler_tsan")
    src = os.path.join(NATIVE, "tests", "sampler_tsan.cpp")
    p = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                        f"-I{os.path.join(NATIVE, 'smi')}", src, "-o", exe], capture_output=True, text=True)
    if p.returncode != 0:
        return p.returncode, p.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    return r.returncode, r.stdout + r.stderr
