"""Lab copy of the kernel library with the opt-in flash-attention backward
variants compiled in (``tools/fa_lab/fa_wave64.inc``: dK/dV with 64 keys per
wave, dQ with 64 queries per wave, D = 128 dK/dV with V in registers).  They
measured 12-50 % slower than the shipped passes (profiles/r5_fa_wave64/), so
the production ``fleetx_amd/_C/_kernels*.so`` does not contain them.

    python tools/fa_lab/build.py            # -> tools/fa_lab/_kernels<EXT>
    FLEETX_KERNELS_LIB=tools/fa_lab/_kernels<EXT> FLEETX_FA_DKDV64=1 python ...

The lab library also carries per-wave ``s_memrealtime`` stamps of the forward
and dK/dV passes (``fa_set_stamps``; read by ``stamp_fwd.py`` /
``stamp_bwd.py``).  ``FX_FA_LAB_DEFS="-DNAME ..."`` builds an experiment
variant named after its defines (e.g. ``-DFA_EXP_NOMASK``: the causal forward
grid with the full tile body, timing only).

Every other object is the production build's (``build/obj``)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from fleetx_amd import _build as B  # noqa: E402


def main():
    B.build_kernels()  # production objects up to date
    kdir = os.path.join(B.CSRC, "kernels")
    inc = os.path.join(HERE, "fa_wave64.inc")
    # FX_FA_LAB_DEFS="-DNAME ...": an experiment build, named after its defines
    defs = os.environ.get("FX_FA_LAB_DEFS", "").split()
    tag = "".join("_" + d[2:].lower() for d in defs)
    obj = os.path.join(HERE, "flash_attn_lab%s.o" % tag)
    src = os.path.join(kdir, "flash_attn.hip")
    if B._newer(obj, [src, inc]):
        B._run([B.hipcc(), "-O3", "-std=c++17", "-fPIC", "--offload-arch=" + B.ARCH,
                "-munsafe-fp-atomics", "-Wno-unused-result", '-DFX_FA_LAB="%s"' % inc]
               + defs + ["-c", src, "-o", obj])
    objs = [os.path.join(B.OBJ, f) for f in sorted(os.listdir(B.OBJ))
            if f.endswith(".o") and f != "flash_attn.hip.o"] + [obj]
    so = os.path.join(HERE, "_kernels" + tag + B.EXT)
    B._run([B.hipcc(), "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-o", so] + objs)
    print(so)


if __name__ == "__main__":
    main()
