"""The optional display: HIP-GL interop entry points of the C-ABI
(bdpt_gl_register_pbo / bdpt_gl_publish / bdpt_gl_unregister, include/bdpt.h) and the X11/GLX
viewer smallpt_gl (csrc/smallpt_gl.c), the counterparts of cudaGLRegisterBufferObject
(smallpt_cpu.c:112-123) and IdleFunc's map / UpdateRendering / unmap (display_func.c:199-215).

No X server or GL-capable display exists here or on the GPU nodes, so the interop itself (a
registered buffer, a mapped copy) is not exercised; what is tested: the entry points refuse
without a current GL context and leave the context usable (rendering afterwards is bit-exact), the
order and argument errors, and that the viewer builds, links and exits cleanly without a display."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import gpu_bidirectional_raytracer_amd as g
import oracle
from conftest import REPO

VIEWER = os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "smallpt_gl")
HAVE_GL_HEADERS = os.path.exists("/usr/include/GL/glx.h") and os.path.exists("/usr/include/X11/Xlib.h")


def _cornell(W, H, device):
    cam, sp = g.default_scene()
    g.update_camera(cam, W, H)
    return g.Renderer(sp, W, H, cam, device=device), cam, sp


def test_gl_entry_points_on_the_cpu_backend():
    """The CPU backend has no device pixels: register refuses with a message, publish before a
    register is an order error, unregister without a buffer is a no-op; the context still renders."""
    r, _, _ = _cornell(33, 25, -1)
    with pytest.raises(g.BdptError) as e:
        r.gl_register_pbo(1)
    assert e.value.code == g._lib.BDPT_EINVAL and "CPU backend" in str(e.value)
    with pytest.raises(g.BdptError) as e:
        r.gl_publish()
    assert e.value.code == g._lib.BDPT_ESTATE and "bdpt_gl_register_pbo" in str(e.value)
    r.gl_unregister()
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    r.path_passes(*s.next(2))
    assert (r.read_radiance()[1] == 2).all()
    r.close()


def test_gl_entry_points_null_context():
    lib = g._lib.lib
    assert lib.bdpt_gl_register_pbo(None, 1) == g._lib.BDPT_EINVAL
    assert lib.bdpt_gl_publish(None) == g._lib.BDPT_EINVAL
    assert lib.bdpt_gl_unregister(None) == g._lib.BDPT_EINVAL


@pytest.mark.skipif(not HAVE_GL_HEADERS, reason="no GL / X11 headers in this image")
def test_viewer_links_and_exits_without_a_display():
    """smallpt_gl resolves libbdpt, libGL and libX11, and with no X display exits with status 2
    before any GPU work (the nodes are headless)."""
    assert os.path.exists(VIEWER), "make builds smallpt_gl when the GL headers are present"
    ldd = subprocess.run(["ldd", VIEWER], capture_output=True, text=True, timeout=30).stdout
    assert "not found" not in ldd, ldd
    for lib in ("libbdpt.so", "libGL.so", "libX11.so"):
        assert lib in ldd, (lib, ldd)
    env = {k: v for k, v in os.environ.items() if k != "DISPLAY"}
    p = subprocess.run([VIEWER, "--frames", "1"], capture_output=True, text=True, timeout=60, env=env,
                       cwd=REPO)
    assert p.returncode == 2, (p.returncode, p.stderr)
    assert "cannot open X display" in p.stderr


def test_viewer_uses_the_interop_entry_points():
    """The viewer hands frames to GL through the C-ABI's interop calls, not a host read-back."""
    src = open(os.path.join(REPO, "gpu_bidirectional_raytracer_amd", "csrc", "smallpt_gl.c")).read()
    for call in ("bdpt_gl_register_pbo", "bdpt_gl_publish", "bdpt_gl_unregister", "GL_PIXEL_UNPACK_BUFFER"):
        assert call in src, call
    assert "bdpt_read_pixels" not in src


@pytest.mark.gpu
def test_gl_register_without_context_leaves_the_context_usable(gpu):
    """On the GPU: with libGL loaded in the process but no current GL context, register refuses
    (BDPT_EINVAL, the context lookup through the loaded library), publish stays an order error,
    and the context renders 4 passes bit-exact against the oracle afterwards."""
    ctypes.CDLL("libGL.so.1")                      # loaded (RTLD_LOCAL), no context made current
    W, H = 65, 49
    r, cam, sp = _cornell(W, H, gpu)
    with pytest.raises(g.BdptError) as e:
        r.gl_register_pbo(1)
    assert e.value.code == g._lib.BDPT_EINVAL and "no OpenGL context" in str(e.value)
    with pytest.raises(g.BdptError) as e:
        r.gl_publish()
    assert e.value.code == g._lib.BDPT_ESTATE
    r.gl_unregister()
    r.light_pass(0)
    s = g.PassScheduler()
    s.light()
    sid, vlp = s.next(4)
    r.path_passes(sid, vlp)
    col, cnt = r.read_radiance()
    rnd = oracle.mt607(0)
    lp = oracle.light_pass(sp, rnd, 0)
    ocol, ocnt, opix = oracle.path_passes(sp, rnd, cam, W, H, lp, sid, vlp)
    assert np.array_equal(col.view(np.uint32), ocol.view(np.uint32))
    assert np.array_equal(cnt, ocnt)
    assert np.array_equal(r.read_pixels(), opix)
    r.close()
