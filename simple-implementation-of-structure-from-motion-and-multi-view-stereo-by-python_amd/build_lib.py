"""Build recipe for libmvs_amd.so (hipcc, gfx950).  Used by __graft_entry__.build().

-ffp-contract=off on both host and device code: the photo test's geometry
reproduces the reference's binary64 operation order; the only fused products
are the ones written as fma() (numpy/OpenBLAS 3-element dot products).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmvs_amd.so")
STAMPS_LIB = os.path.join(HERE, "libmvs_amd_stamps.so")   # diagnostic build (-DMVS_STAMPS)
ASAN_LIB = os.path.join(HERE, "libmvs_amd_asan.so")       # host code under ASan + UBSan (tools/asan_cpu.sh)
SOURCES = ["mvs_kernels.hip", "mvs_score_tab.hip", "sfm_kernels.hip", "mvs_engine.cpp"]
HEADERS = ["mvs_internal.h", "mvs_device.h", "mvs_mma.h", os.path.join("..", "..", "include", "mvs_amd.h")]
OBJDIR = os.path.join(HERE, "build")   # per-source objects (git- and gpurun-ignored)
ARCH = os.environ.get("MVS_OFFLOAD_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force=False, verbose=False, stamps=False, asan=False):
    out = STAMPS_LIB if stamps else ASAN_LIB if asan else LIB
    if not stamps and not asan and not force and not needs_build():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           # no wave-aggregated global atomics: their immediate wait on the
           # return value would also drain the scorer's LDS-DMA prefetch
           "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function"]
    if stamps:
        cmd.append("-DMVS_STAMPS")
        # diagnostic A/B switches for the stamps build, e.g. MVS_STAMPS_DEFS=MVS_DIAG_NOSTORE
        cmd += [f"-D{d}" for d in os.environ.get("MVS_STAMPS_DEFS", "").split()]
    if asan:
        # the host code only (the engine's commit, seeding, filter, sort
        # bookkeeping, C-ABI checks); device code is never sanitized here
        for f in ("-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                  "-fno-omit-frame-pointer", "-shared-libsan", "-g"):
            cmd += ["-Xarch_host", f]
    # A/B of code-generation options (e.g. "-mllvm -amdgpu-sched-strategy=iterative-ilp")
    cmd += os.environ.get("MVS_EXTRA_FLAGS", "").split()
    # one object per source, compiled in parallel, then linked
    tag = "stamps" if stamps else "asan" if asan else "lib"
    os.makedirs(OBJDIR, exist_ok=True)
    objs = [os.path.join(OBJDIR, f"{tag}_{f}.o") for f in SOURCES]
    procs = []
    for f, o in zip(SOURCES, objs):
        c = cmd + ["-c", os.path.join(CSRC, f), "-o", o]
        if verbose:
            print(" ".join(c), file=sys.stderr)
        procs.append(subprocess.Popen(c, cwd=CSRC))
    bad = [f for f, p in zip(SOURCES, procs) if p.wait() != 0]
    if bad:
        raise subprocess.CalledProcessError(1, f"hipcc {bad}")
    # the link takes the compile options minus the "-mllvm X" pairs (removed
    # pairwise: a bare X left behind would be an unknown argument)
    link = []
    k = 0
    while k < len(cmd):
        if cmd[k] == "-mllvm":
            k += 2
            continue
        link.append(cmd[k])
        k += 1
    link += ["-shared", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.check_call(link, cwd=CSRC)
    check_undefined(out + ".tmp")
    os.replace(out + ".tmp", out)
    return out


def check_undefined(path):
    """A kernel template whose body the host pass rejects without a
    diagnostic leaves its launch stub undefined: the .so links, then fails to
    load.  Refuse such a build here."""
    nm = "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(nm):
        return
    undef = subprocess.run([nm, "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    bad = [ln.split()[-1] for ln in undef.splitlines() if "_GLOBAL__N_" in ln]
    if bad:
        os.remove(path)
        raise RuntimeError(f"{len(bad)} kernel(s) of this build have no host stub, e.g. {bad[0]}")


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, stamps="--stamps" in sys.argv,
                asan="--asan" in sys.argv))
