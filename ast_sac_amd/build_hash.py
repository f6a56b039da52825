"""Content hash of the native sources: __graft_entry__.build() compiles it into each library
(shipsim_build_info / sacf_build_info) and rebuilds whenever it changes; the ctypes bindings refuse a
library whose embedded hash differs from the sources next to it (a stale build)."""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)

SOURCES = {
    "shipsim": ["ast_sac_amd/csrc/shipsim_kernels.hip", "ast_sac_amd/csrc/shipsim_device.hpp",
                "ast_sac_amd/csrc/shipsim_diag.hpp", "include/shipsim.h"],
    "sacfused": ["ast_sac_amd/csrc/sac_kernels.hip", "include/sac_fused.h"],
}


# code-generation flags of both libraries (include paths are added by the build and not hashed, so the
# hash is the same in every checkout of the same sources)
HIPFLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared", "-std=c++17"]
# per-library additions. shipsim (object 1, below): no machine-level loop-invariant code motion — hoisting the tick loop's
# constants (fp64 literals, addresses) out of the 4096-tick loop held them in registers for the whole
# launch: 256 VGPR + 161 AGPR and 55 SGPR spill lanes in the headline kernel, against 256 + 46 and none
# without it, at the same speed. And the machine scheduler's max-ILP strategy instead
# of the occupancy-first default: the step kernels run one wave per SIMD whatever the schedule, so interleaving
# independent FP64 chains is what shortens the tick (+0.7 % on the headline, spill-free; profiles/round4/
# r4z_sched_ab.txt), with the scheduler's AMDGPU register-pressure trackers (+0.5 %, r4zz_sched3_ab.txt).
LIB_FLAGS = {"shipsim": ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-mllvm", "-amdgpu-use-amdgpu-trackers"],
             "sacfused": []}
# libraries built from several objects of the same source, each with flags of its own (then linked into one .so).
# sacfused: max-ILP is 0.6 µs faster per grad step at H = 256 but spills SGPRs in three kernels at H = 448 / 512,
# so the widths up to 384 (and the C ABI) are one object with it and the two widest another without
# (sac_kernels.hip SACF_TU).
# shipsim: the C2 three-wave kernel (its own object, SHIPSIM_TU 2) keeps machine LICM — its loops have registers to
# spare, and hoisting the fp64 constants of atan / sincos out of the tick loop shortens the tick; every other kernel
# and the C ABI are the object without it (SHIPSIM_TU 1).
OBJECTS = {"sacfused": [["-DSACF_TU=1", "-mllvm", "-amdgpu-sched-strategy=max-ilp"], ["-DSACF_TU=2"]],
           "shipsim": [["-DSHIPSIM_TU=1", "-mllvm", "-disable-machine-licm"], ["-DSHIPSIM_TU=2"]]}


def lib_flag_sets(lib):
    """The flag sets the library is compiled with: one per object (one set for a single-object library)."""
    return [LIB_FLAGS[lib] + extra for extra in OBJECTS.get(lib, [[]])]


def source_hash(lib):
    h = hashlib.sha256()
    for rel in SOURCES[lib]:
        with open(os.path.join(_ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read() + b"\0")
    for flags in lib_flag_sets(lib):
        h.update(" ".join(HIPFLAGS + flags).encode() + b"\0")
    return h.hexdigest()[:16]


def check_library(lib, info, path, explicit):
    """Raise if the library at `path` (build info string `info`) was not built from these sources."""
    want = source_hash(lib)
    if info.split()[-1] != want and not explicit:
        raise RuntimeError(f"{path} was built from other sources ({info!r}, sources hash {want}): rebuild with "
                           f"python -c 'import __graft_entry__ as g; g.build()'")
