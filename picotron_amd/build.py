"""Build the gfx950 kernels into one in-tree shared library: picotron_amd/lib/libpicotron_hip.so.

Each csrc/*.hip is compiled with hipcc --offload-arch=gfx950 (cross-compiles without a GPU) in
parallel, then linked.  The library is linked against torch's bundled libamdhip64 (RUNPATH ->
torch/lib first): torch loads its HIP runtime before we dlopen ours, the shared SONAME
(libamdhip64.so.7) resolves to that one copy, and streams / device pointers from torch are
valid in our calls (one HIP runtime per process).
"""
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libpicotron_hip.so")
ARCH = "gfx950"


def _torch_lib_dir():
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


# per-source code-generation flags.  attention: MFMA results in VGPRs (gfx950's unified register
# file) instead of AGPRs -- the softmax reads every S / dP accumulator, and the AGPR form cost a
# v_accvgpr_read per element plus registers (fwd 156 -> 124 VGPRs: 3 -> 4 waves per SIMD).
FILE_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def _compile(src, obj, extra):
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", src, "-o", obj,
           "-Wno-unused-result"] + FILE_FLAGS.get(os.path.basename(src), []) + extra
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {os.path.basename(src)}:\n{r.stderr}")
    return obj


def build(force=False, verbose=True, extra=(), out=None):
    """out: another library path (A/B and diagnostic builds with `extra` flags; always rebuilt)."""
    if out is not None:
        force = True
    lib_path = out or LIB
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sources()
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    newest = max(os.path.getmtime(p) for p in srcs + hdrs + [__file__])
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        if verbose:
            print(f"[picotron_amd.build] up to date: {LIB}")
        return LIB
    objdir = os.path.join(LIBDIR, "obj" if out is None else "obj_alt")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s)[:-4] + ".o") for s in srcs]
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda so: _compile(so[0], so[1], list(extra)), zip(srcs, objs)))
    tl = _torch_lib_dir()
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path + ".tmp"] + objs + \
          [f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(lib_path + ".tmp", lib_path)
    if verbose:
        print(f"[picotron_amd.build] built {lib_path} from {len(srcs)} sources")
    return lib_path


if __name__ == "__main__":
    # python -m picotron_amd.build [--force] [--out PATH -DFLAG ...]  (--out: an A/B or diagnostic build)
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else None
    flags = [a for a in args if a.startswith("-D")]
    build(force="--force" in args, extra=flags, out=os.path.abspath(out) if out else None)
