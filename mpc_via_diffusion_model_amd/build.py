"""Build libmpcd.so in-tree with hipcc for gfx950 (no torch extension machinery, no JIT cache).

    python -m mpc_via_diffusion_model_amd.build        # or __graft_entry__.build()

Every translation unit is compiled with -ffp-contract=off: the denoise update and the fp64
rollout must round each product separately, exactly as the reference's torch / numpy code does.
"""
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "libmpcd.so")
OBJ = os.path.join(PKG, "_build")
ARCH = os.environ.get("MPCD_OFFLOAD_ARCH", "gfx950")
SOURCES = ["mpcd_api.hip", "comm.hip", "mlp_sampler.hip", "mlp_x3.hip", "mlp_rw.hip", "mlp_h2.hip", "cond_prologue.hip", "rollout.hip", "unet.hip", "unet_mx.hip", "unet_fused.hip", "train.hip"]
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs (no v_accvgpr_read before every epilogue op;
# f32 MFMA and VALU share issue on gfx950, so those moves cost MFMA time).
# per-source additions. mlp_x3.hip: the memory-clause machine scheduler groups each layer's weight / LDS
# fragment loads ahead of the MFMA chains (measured: cfg2 sampler 1.243 -> 1.205 ms; no effect on unet_mx)
SOURCE_FLAGS = {"mlp_x3.hip": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]}
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}", "-mllvm", "-amdgpu-mfma-vgpr-form", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable"]


ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
LIBS = [f"-L{ROCM_LIB}", "-lrccl", f"-Wl,-rpath,{ROCM_LIB}"]  # RCCL: the C ABI's candidate-batch exchange


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libmpcd.so)")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, variant=None, defines=()):
    """variant: build an experiment copy (libmpcd_<variant>.so, objects in _build_<variant>/) with
    extra -D defines; load it with MPCD_LIB=<path>. The default build is the product library."""
    cc = hipcc()
    out, obj, flags, extra = OUT, OBJ, list(FLAGS), []
    if variant:
        out = os.path.join(PKG, f"libmpcd_{variant}.so")
        obj = OBJ + "_" + variant
        # MPCD_VARIANT: the wrong-result timing switches of the kernels compile only in such a build
        flags += ["-DMPCD_VARIANT"] + [f"-D{d}" for d in defines]
        # experiment builds only: MPCD_DROP_FLAGS / MPCD_EXTRA_FLAGS (space separated) edit the compile line
        drop = os.environ.get("MPCD_DROP_FLAGS", "").split()
        for f in drop:
            while f in flags:
                i = flags.index(f)
                del flags[i]
                if i > 0 and flags[i - 1] == "-mllvm":
                    del flags[i - 1]
        extra = os.environ.get("MPCD_EXTRA_FLAGS", "").split()  # appended last (after SOURCE_FLAGS)
    os.makedirs(obj, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(os.path.dirname(PKG), "include", "mpcd.h"))
    jobs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj, src.replace(".hip", ".o"))
        if force or _stale(o, [s] + headers):
            jobs.append([cc] + flags + SOURCE_FLAGS.get(src, []) + extra + ["-c", s, "-o", o])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr:
            sys.stderr.write(r.stderr)

    with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8) or 1) as ex:
        list(ex.map(run, jobs))
    objs = [os.path.join(obj, s.replace(".hip", ".o")) for s in SOURCES]
    if force or jobs or _stale(out, objs):
        tmp = out + ".tmp"  # link beside, then rename: a reader never sees a half-written library
        run([cc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp] + objs + LIBS)
        os.replace(tmp, out)
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--force"]
    variant = args[0] if args else None
    print(build(force="--force" in sys.argv, verbose=True, variant=variant, defines=args[1:]))
