"""Build libnais_hip.so in-tree for gfx950 (hipcc; no torch extension machinery needed)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("nais_kernels.hip", "nais_train.hip", "nais_new4.hip", "nais_pairs.hip", "nais_dot.hip", "nais_disent.hip", "nais_generic.hip")]
SRC = SRCS[0]
OUT = os.path.join(HERE, "libnais_hip.so")
ARCH = os.environ.get("NAIS_OFFLOAD_ARCH", "gfx950")


# nais_kernels.hip: MFMAs in their VGPR form (accumulators in VGPRs, not AGPRs), so an epilogue
# reads its accumulator values without a v_accvgpr_read each. (Introduced for the round-3 x3c
# pair-table A/B, since removed; the remaining kernels compiled to the same VGPR / AGPR counts
# either way.)
PER_SRC = {"nais_kernels.hip": ("-mllvm", "-amdgpu-mfma-vgpr-form=1")}


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


OBJDIR = os.path.join(ROOT, "build_obj")   # per-translation-unit object cache (git- and gpurun-ignored)


def build(force=False, extra=(), out=None, extra_for=None, replace=None):
    """Compile the kernels into OUT (or `out`, e.g. an A/B variant with extra -D flags). Objects are
    cached per (translation unit, flags) under build_obj/: a TU is recompiled only when it or a
    header is newer than its object, so an edit to one .hip file (or an A/B -D flag that one TU
    reads, passed through `extra_for` = {basename: flags}) recompiles that file alone. `replace` =
    {basename: path} compiles another source in that TU's place (a probe build that includes the
    product source, e.g. scripts/probes/train_timing.hip) -- never for the product library."""
    if replace and out is None:
        raise ValueError("replace= builds a variant: give it out=")
    import hashlib
    OUT_ = out or OUT
    csrc = os.path.join(HERE, "csrc")
    headers = [os.path.join(ROOT, "include", "nais.h"),
               *(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".h"))]
    hdr_time = max(os.path.getmtime(h) for h in headers)
    # -fno-slp-vectorize: hipcc's SLP pass packs adjacent f32 adds/muls into v_pk_*_f32, which
    # cost more issue slots than two scalar ops beside MFMAs (cdna_hip_programming.md, price table);
    # measured +5 % on the split-fp16 catalog kernel (profiles/r1/ab_*.json).
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize",
             "-I", os.path.join(ROOT, "include"), *extra]
    os.makedirs(OBJDIR, exist_ok=True)
    objs, todo = [], []
    for src in SRCS:
        base = os.path.basename(src)
        f = [*flags, *PER_SRC.get(base, ()), *(extra_for or {}).get(base, ())]
        newest = max(os.path.getmtime(src), hdr_time)
        if replace and base in replace:
            src = os.path.abspath(replace[base])
            f = [*f, "-DNAIS_PROBE_SOURCE=" + os.path.basename(src)]
            newest = max(newest, os.path.getmtime(src))
        key = hashlib.sha1(" ".join(f).encode()).hexdigest()[:12]
        o = os.path.join(OBJDIR, f"{base}.{key}.o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < newest:
            todo.append((src, o, f))
    # the link is keyed too: a sidecar next to the library records the objects it was linked
    # from (their names carry the flag hashes), so a variant name reused with other -D flags, or
    # a library linked from other objects, is relinked even when it is newer than the objects
    stamp = OUT_ + ".objs"
    linked = open(stamp).read() if os.path.exists(stamp) else None
    if (not todo and os.path.exists(OUT_) and linked == "\n".join(objs)
            and all(os.path.getmtime(OUT_) >= os.path.getmtime(o) for o in objs)):
        return OUT_
    # the changed translation units compiled in parallel, then one link; temporary names carry
    # the pid, so concurrent builds with the same flags do not write the same file
    tmp = f".{os.getpid()}.tmp"
    procs = [(subprocess.Popen([hipcc(), *f, "-c", "-o", o + tmp, src], stdout=subprocess.PIPE,
                               stderr=subprocess.STDOUT, text=True), src, o) for src, o, f in todo]
    failed = []
    for pr, src, o in procs:
        log, _ = pr.communicate()
        if pr.returncode != 0:
            sys.stderr.write(log)
            failed.append(os.path.basename(src))
        else:
            os.replace(o + tmp, o)
    if failed:
        raise RuntimeError(f"hipcc failed on {failed}")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT_ + tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"hipcc link failed ({r.returncode}): {' '.join(cmd)}")
    os.replace(OUT_ + tmp, OUT_)
    with open(stamp + tmp, "w") as fh:
        fh.write("\n".join(objs))
    os.replace(stamp + tmp, stamp)
    return OUT_


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
