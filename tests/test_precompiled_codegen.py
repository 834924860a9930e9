"""Spill guard for the precompiled kernels inside libbdpt.so (the instances that run when the
scene-specialised build is off or unavailable, and the BVH instance N = -1 that always runs for
large scenes).  The gfx950 code object is unpacked from the library's .hip_fatbin section and its
kernel metadata read; every instance's VGPR spills, scratch size and SGPR spills must equal the
recorded values below, so a register-pressure regression fails here on the CPU instead of showing
up as a slower kernel on the GPU.  (tests/test_jit_codegen.py guards the specialised builds.)

Recorded values and why they are acceptable:
  * no instance spills VGPRs or uses scratch (private segment 0) -- including the BVH instance,
    which earlier builds ran with 10 spilled VGPRs;
  * the per-N instances hold the scene geometry in SGPRs (wave-uniform constant loads); from
    N = 12 spheres (fused) / 13 (pass streams) the SGPR file (106) overflows and the excess goes to
    VGPR lanes (v_writelane / v_readlane, no memory traffic): fused 2 per sphere above 11, pass
    streams 2, 3, 6, 7, 9 for N = 12..16 (from N = 11, 2 per sphere above 10, before the VLP-only
    shadow rounds skipped the emitters, BDPT_VAC_SKIP, and the lane-group rule BDPT_LG_RULE).  These instances only run with
    specialisation off: by default a <= 64-sphere scene runs its hipRTC build;
  * the BVH instance keeps its traversal state in SGPRs and moves 10 (pass streams) / 2 (fused)
    of them to VGPR lanes in the same way (11 / 3 before round 4's settled pass-stream randoms
    and buffer-descriptor table loads; 8 / 6 before round 3's grouped path regeneration and
    paired random loads; 10 / 15 before the pass table of short calls moved into the kernel
    arguments).
"""
import os
import subprocess
import sys

import pytest

from conftest import REPO

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "libbdpt.so")
sys.path.insert(0, os.path.join(REPO, "tools"))


def _sgpr_spills(n, streams):
    if n == -1:
        return 11 if streams else 2   # (streams: 10 before the d_scp descriptor, BDPT_SCP)
    if streams:
        return {12: 2, 13: 3, 14: 6, 15: 7, 16: 9}.get(n, 0)
    return 2 * (n - 11) if n > 11 else 0


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    if not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("no ROCm LLVM tools")
    import jit_codegen_check as jc
    d = tmp_path_factory.mktemp("co")
    fat, co = str(d / "fat.bin"), str(d / "co.o")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", LIB,
                           str(d / "stripped.so")])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co], text=True)
    return {k["name"]: k for k in jc.kernel_notes(notes)}


def test_every_instance_is_present(kernels):
    for st in (0, 1):
        for n in list(range(0, 17)) + [-1]:
            name = f"_Z18bdpt_path_kernel_tIL{'i' if n >= 0 else 'in'}{abs(n)}ELb{st}EEv14bdpt_path_args"
            assert name in kernels, name
    for k in ("bdpt_mt607_kernel", "bdpt_light_kernel", "bdpt_accum_kernel", "bdpt_rand_planar_kernel",
              "bdpt_sincos_planar_kernel",
              "bdpt_pixels_kernel", "bdpt_frame_add_kernel"):
        assert k in kernels, k


def test_no_vgpr_spills_or_scratch(kernels):
    for name, k in kernels.items():
        assert k["vgpr_spill_count"] == 0, k
        assert k["private_segment_fixed_size"] == 0, k


def test_sgpr_spills_match_record(kernels):
    for st in (0, 1):
        for n in list(range(0, 17)) + [-1]:
            name = f"_Z18bdpt_path_kernel_tIL{'i' if n >= 0 else 'in'}{abs(n)}ELb{st}EEv14bdpt_path_args"
            assert kernels[name]["sgpr_spill_count"] == _sgpr_spills(n, st), kernels[name]
    for k in ("bdpt_mt607_kernel", "bdpt_light_kernel", "bdpt_accum_kernel"):
        assert kernels[k]["sgpr_spill_count"] == 0, kernels[k]


def test_occupancy_of_the_path_instances(kernels):
    """Every pass-stream per-N instance fits 6 waves/SIMD (<= 80 VGPRs, 512 / 6 rounded down to 8);
    the fused instances are bounded at 5 (BDPT_FUSED_WAVES, <= 96: their LDS holds a CU at 5
    workgroups anyway, and round 3's grouped regeneration and paired random loads use the room);
    the BVH instances fit 5 (<= 96)."""
    for st in (0, 1):
        for n in list(range(0, 17)) + [-1]:
            name = f"_Z18bdpt_path_kernel_tIL{'i' if n >= 0 else 'in'}{abs(n)}ELb{st}EEv14bdpt_path_args"
            bound = 96 if (n == -1 or not st) else 80
            assert kernels[name]["vgpr_count"] <= bound, kernels[name]
