"""The C-ABI library loads and exports every symbol include/semtsdf.h declares (no GPU
compute is called here)."""
import os
import re

from conftest import ROOT


def declared():
    with open(os.path.join(ROOT, "include", "semtsdf.h")) as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(semtsdf_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    from semtsdf import _lib as L

    names = declared()
    assert len(names) >= 30
    assert set(names) == set(L.SIGNATURES), set(names) ^ set(L.SIGNATURES)


def test_library_exports_every_symbol():
    from semtsdf import _lib as L

    lib = L.load()
    for n in declared():
        assert hasattr(lib, n), n
    assert lib.semtsdf_abi_version() == 12
    key = lib.semtsdf_build_key().decode()
    assert len(key) == 64 and int(key, 16) >= 0  # the sha-256 build key (__graft_entry__.build_key)


def test_structs_match_header_sizes():
    import ctypes as C

    from semtsdf import _lib as L

    # semtsdf_params: 3 i32 + 13 f32 + 32 f32 + 2 i32 + 5 f32 + u32 + 3 i32
    assert C.sizeof(L.Params) == 4 * (3 + 9 + 1 + 32 + 2 + 5 + 1 + 3)
    assert C.sizeof(L.AssocStats) == 4 * (2 + 32 + 32) + 256 + 4 + 4
    # semtsdf_state: u32 n_obs, i32 num_objs, 3 i32 local_dim (+ 4 B padding), 3 u64
    assert C.sizeof(L.State) == 4 * 5 + 4 + 8 * 3
    # semtsdf_timing: 18 fields of 8 bytes (doubles or u64)
    assert C.sizeof(L.Timing) == 8 * 18


def test_argument_errors_without_a_device():
    """Argument checks of the ABI 8 entry points return errors (and a message) before any
    GPU work: NULL handles/pointers, misaligned kernel copies, bad memcpy kinds."""
    import ctypes as C

    from semtsdf import _lib as L

    lib = L.load()
    E = (C.c_float * 16)()
    s2w = (C.c_float * 16)()
    c = (C.c_float * 3)()
    buf = C.c_void_p(0x1000)
    rc = lib.semtsdf_parse_frame_view_dev(None, buf, buf, buf, E, s2w, c, L.RENDER_LABEL, buf, None, None)
    assert rc != 0 and b"NULL" in lib.semtsdf_last_error()
    # kernel copy (kind 4): 16-B alignment of both pointers and the size is checked first
    rc = lib.semtsdf_memcpy(C.c_void_p(0x1004), C.c_void_p(0x2000), 64, 4, None)
    assert rc != 0 and b"16-B" in lib.semtsdf_last_error()
    rc = lib.semtsdf_memcpy(C.c_void_p(0x1000), C.c_void_p(0x2000), 40, 4, None)
    assert rc != 0 and b"16-B" in lib.semtsdf_last_error()
    rc = lib.semtsdf_memcpy(C.c_void_p(0x1000), C.c_void_p(0x2000), 64, 7, None)
    assert rc != 0 and b"kind" in lib.semtsdf_last_error()
    # ABI 9: the decision on given inputs, the libm check, the sharded exact path
    rc = lib.semtsdf_filter_overlaps_dev(None, buf, buf, buf, None, None)
    assert rc != 0 and b"NULL" in lib.semtsdf_last_error()
    rc = lib.semtsdf_libm_eval(2, buf, buf, 16, None)
    assert rc != 0 and b"fn" in lib.semtsdf_last_error()
    rc = lib.semtsdf_shard_assoc_pixels(None, buf, buf, None)
    assert rc != 0 and b"NULL" in lib.semtsdf_last_error()
    rc = lib.semtsdf_shard_assoc_apply_exact(None, buf, buf, buf, None, None)
    assert rc != 0 and b"NULL" in lib.semtsdf_last_error()


def test_params_validation_without_a_device():
    """semtsdf_create validates the parameters before touching a device: the association's prior
    must lie in [2^-10, 1) (the range its f32 rule is evaluated for)."""
    import ctypes as C

    from semtsdf import _lib as L

    lib = L.load()
    p = L.Params()
    intr = (C.c_float * 4)(520.9, 521.0, 325.1, 249.7)
    assert lib.semtsdf_params_default(C.byref(p), 32, intr, 64, 48) == 0
    for a in range(3):
        p.voxel[a] = 0.01
    p.mu = 0.05
    for bad in (0.0, -0.05, 1.0, 2.0, float("nan"), 2.0 ** -11):
        p.prior_mrcnn_err_rate = bad
        h = C.c_void_p()
        rc = lib.semtsdf_create(C.byref(p), 0, C.byref(h))
        assert rc == L.ERR_INVALID and b"prior_mrcnn_err_rate" in lib.semtsdf_last_error(), bad


def test_detector_library_exports_every_symbol():
    """include/semtsdf_det.h (the Mask R-CNN producer's NMS, libsemtsdf_det.so): every declared symbol
    exported; argument errors refused without touching a device."""
    import ctypes as C

    with open(os.path.join(ROOT, "include", "semtsdf_det.h")) as f:
        txt = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(semtsdf_det_[a-z0-9_]+)\s*\(", txt)))
    assert names == ["semtsdf_det_abi_version", "semtsdf_det_nms", "semtsdf_det_nms_workspace", "semtsdf_det_roi_align"]
    lib = C.CDLL(os.path.join(ROOT, "slam-maskrcnn_amd", "semtsdf", "libsemtsdf_det.so"))
    for n in names:
        assert hasattr(lib, n), n
    assert lib.semtsdf_det_abi_version() == 2
    lib.semtsdf_det_nms_workspace.restype = C.c_size_t
    assert lib.semtsdf_det_nms_workspace(6000) == 6000 * 94 * 8
    lib.semtsdf_det_nms.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p]
    assert lib.semtsdf_det_nms(None, 16385, 0.5, 10, None, None, None, None) == 1  # too many boxes, NULLs
    assert lib.semtsdf_det_nms(None, -1, 0.5, 10, None, None, None, None) == 1
