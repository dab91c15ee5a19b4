#!/usr/bin/env python3
"""Native build for the gfx950 kernels and the C++ runtime pieces.

Generates a ninja file and builds, in-tree (so the .so files travel to the GPU
box with the repo snapshot):

  * ``<pkg>/_native/libshai_kernels.so`` -- HIP kernels (hipcc --offload-arch=gfx950)
    plus the torch operator registrations (``torch.ops.shai.*``).
  * ``<pkg>/_native/libshai_runtime.so`` -- host C++ runtime (paged-KV block
    manager, batching scheduler helpers) exposed through a C ABI (ctypes).
  * ``<pkg>/_native/libshai_comm.so`` -- xGMI peer-to-peer all-reduce (HIP IPC).

Kernel translation units include no torch headers, so editing a kernel
recompiles in seconds; only ``bindings.cpp`` pulls in ATen.

Usage: python csrc/build.py [--clean] [-j N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "scalable-hw-agnostic-inference_amd")
OUT = os.path.join(PKG, "_native")
BUILD = os.path.join(ROOT, "build", "native")
# device debug flavour (--debug / build(debug=True)): -DSHAI_KERNEL_DEBUG (device bounds asserts on DMA offsets, LDS
# indices and slot ids in the hand-scheduled kernels; hazard-safe waits: counted vmcnt -> vmcnt(0), wider s_nop
# margins), built into its own directories; SHAI_KERNEL_DEBUG=1 makes shai_amd.native load it
OUT_DEBUG = os.path.join(PKG, "_native_debug")
BUILD_DEBUG = os.path.join(ROOT, "build", "native_debug")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

KERNEL_SRCS = ["kernels/norm.hip", "kernels/gemm.hip", "kernels/gemm_lds.hip", "kernels/gemm_8ph.hip", "kernels/gemm_w4.hip", "kernels/gemm_ws.hip", "kernels/conv_halo.hip", "kernels/attention.hip", "kernels/attention2.hip", "kernels/attention3.hip", "kernels/elementwise.hip", "kernels/dit.hip",
               "kernels/sampling.hip", "kernels/gemv.hip", "kernels/gemv2.hip",
               "kernels/gemm_f8.hip"]
# per-source extra hipcc flags: gemm_w4's epilogue (256 accumulators x an activation) is larger than LLVM's
# default pragma-unroll budget; partially unrolled it would index the accumulators at run time (scratch)
EXTRA_KFLAGS = {"kernels/attention3.hip": "-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize",
                # flash2 (d128): +0.5-1.2 % at the Flux / LLM-prefill shapes with the same flags (attention lab A/B)
                "kernels/attention2.hip": "-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize",
                "kernels/gemm_w4.hip": "-mllvm -pragma-unroll-threshold=100000",
                "kernels/gemm_ws.hip": "-mllvm -pragma-unroll-threshold=100000 -fno-slp-vectorize",
                "kernels/conv_halo.hip": "-mllvm -pragma-unroll-threshold=100000 -fno-slp-vectorize"}
BINDING_SRCS = ["bindings.cpp"]
RUNTIME_SRCS = ["runtime/block_manager.cpp", "runtime/scheduler.cpp"]
COMM_SRCS = ["comm/p2p_allreduce.hip"]


def torch_paths():
    import torch  # noqa: F401  (only for include/lib dirs)
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames else ce.include_paths(True)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def write_ninja(path: str, out: str = OUT, build_dir: str = BUILD, debug: bool = False) -> dict:
    inc, tlib, abi = torch_paths()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    kflags = f"--offload-arch={ARCH} -O3 -std=c++17 -fPIC -ffp-contract=fast -Wno-unused-result -I{CSRC}"
    if debug:
        kflags += " -DSHAI_KERNEL_DEBUG"
    incs = " ".join(f"-isystem {p}" for p in inc)
    bflags = (f"-O2 -std=c++17 -fPIC -D_GLIBCXX_USE_CXX11_ABI={abi} -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 "
              f"-I{CSRC} {incs} -isystem {ROCM}/include -Wno-deprecated-declarations")
    rflags = f"-O3 -std=c++17 -fPIC -Wall -I{CSRC}"
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"kflags = {kflags}",
        f"bflags = {bflags}",
        f"rflags = {rflags}",
        # compiler depfiles (-MD -MF): an edit to ANY included header (gemm_epilogue.h, ...) rebuilds its users
        "rule hip",
        "  command = $hipcc $kflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule cxx",
        "  command = c++ $bflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule rcxx",
        "  command = c++ $rflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link_kernels",
        f"  command = $hipcc --offload-arch={ARCH} -shared -fPIC $in -o $out -L{tlib} -Wl,-rpath,{tlib} "
        f"-lc10 -lc10_hip -ltorch_cpu -ltorch_hip -L{ROCM}/lib -lamdhip64",
        "  description = LINK $out",
        "rule link_hip",
        f"  command = $hipcc --offload-arch={ARCH} -shared -fPIC $in -o $out -L{ROCM}/lib -lamdhip64",
        "  description = LINK $out",
        "rule link_cxx",
        "  command = c++ -shared -fPIC $in -o $out -lpthread",
        "  description = LINK $out",
    ]
    targets = {}

    def objs(srcs, rule):
        out = []
        for s in srcs:
            if not os.path.exists(os.path.join(CSRC, s)):
                continue
            o = os.path.join(build_dir, s.replace("/", "_") + ".o")
            lines.append(f"build {o}: {rule} {os.path.join(CSRC, s)} | {os.path.join(CSRC, 'kernels', 'common.h')} "
                         f"{os.path.join(CSRC, 'kernels', 'launchers.h')}")
            if s in EXTRA_KFLAGS:
                lines.append(f"  kflags = $kflags {EXTRA_KFLAGS[s]}")
            out.append(o)
        return out

    k = objs(KERNEL_SRCS, "hip") + objs(BINDING_SRCS, "cxx")
    targets["kernels"] = os.path.join(out, "libshai_kernels.so")
    lines.append(f"build {targets['kernels']}: link_kernels {' '.join(k)}")
    r = objs(RUNTIME_SRCS, "rcxx")
    if r:
        targets["runtime"] = os.path.join(out, "libshai_runtime.so")
        lines.append(f"build {targets['runtime']}: link_cxx {' '.join(r)}")
    c = objs(COMM_SRCS, "hip")
    if c:
        targets["comm"] = os.path.join(out, "libshai_comm.so")
        lines.append(f"build {targets['comm']}: link_hip {' '.join(c)}")
    lines.append("default " + " ".join(targets.values()))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return targets


LAST_BUILD: dict = {}


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False, debug: bool = False) -> dict:
    out, bdir = (OUT_DEBUG, BUILD_DEBUG) if debug else (OUT, BUILD)
    if clean and os.path.isdir(bdir):
        shutil.rmtree(bdir)
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(out, exist_ok=True)
    ninja_file = os.path.join(bdir, "build.ninja")
    targets = write_ninja(ninja_file, out, bdir, debug)
    ninja = shutil.which("ninja")
    if ninja is None:
        import ninja as _nj  # pip package ships the binary
        ninja = os.path.join(_nj.BIN_DIR, "ninja")
    cmd = [ninja, "-f", ninja_file]
    if jobs:
        cmd += ["-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd, cwd=bdir, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    sys.stdout.write(r.stdout)
    if r.returncode != 0:
        raise subprocess.CalledProcessError(r.returncode, cmd, r.stdout)
    # what ninja actually did: "[i/n] HIP <src>" per compiled object, "no work to do" when all were reused
    compiled = [ln.split("] ", 1)[1].split(" ", 1)[1] for ln in r.stdout.splitlines()
                if ln.startswith("[") and ("] HIP " in ln or "] CXX " in ln)]
    LAST_BUILD.clear()
    LAST_BUILD.update(compiled=compiled, linked=sum("] LINK " in ln for ln in r.stdout.splitlines()),
                      up_to_date="no work to do" in r.stdout)
    return targets


def summary() -> str:
    """One line: whether the last build() compiled objects or reused every one of them."""
    if not LAST_BUILD:
        return "native build: not run"
    if LAST_BUILD["up_to_date"]:
        return "native build: up to date (all objects reused)"
    return (f"native build: compiled {len(LAST_BUILD['compiled'])} object(s), relinked {LAST_BUILD['linked']} "
            f"librar{'y' if LAST_BUILD['linked'] == 1 else 'ies'}: " + ", ".join(
                os.path.relpath(c, CSRC) if os.path.isabs(c) else c for c in LAST_BUILD["compiled"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(16, os.cpu_count() or 8))
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--debug", action="store_true", help="device debug flavour into _native_debug/")
    a = ap.parse_args()
    t = build(a.clean, a.j, a.v, a.debug)
    for k, v in t.items():
        print(f"{k}: {v}")
    print(summary())


if __name__ == "__main__":
    sys.exit(main())
