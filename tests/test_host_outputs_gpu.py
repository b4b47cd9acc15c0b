"""Zero-copy outputs into CALLER buffers on the reference-compatible run_host path: a caller
array passed again for a second frame is mapped for the GPU (hipHostRegister) and the frame graph's reprojection
writes the disparity and the cloud into it directly, exactly as into the engine's own pinned buffers.  Reuse, swap
and swap-back of the buffers must give the same bytes as the pinned-I/O path, and a buffer the caller stopped passing
must not be written any more."""
import numpy as np
import pytest
import torch

from stereoalgorithms_amd import _native as N
from stereoalgorithms_amd.utils.synthetic import batch_pairs

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (torch.cuda.is_available() and N.available()), reason="needs GPU + native lib")]

Q = np.array([[1, 0, 0, -320.0], [0, 1, 0, -240.0], [0, 0, 0, 500.0], [0, 0, 1 / 60.0, 0]], np.float32)


def test_caller_buffers_reuse_and_swap():
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    e = NativeStereoEngine("raftstereo-realtime", None, 480, 640, batch=1, device=0)
    e.set_Q(Q)
    l, r = batch_pairs(1, 480, 640, seed=3)
    hb = e.host_buffers()
    hb["left"][...] = l
    hb["right"][...] = r
    e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
    ref_d, ref_c = hb["disp"].copy(), hb["cloud"].copy()
    hb = None
    d1, c1 = np.full((1, 480, 640), -7.0, np.float32), np.full((1, 480, 640, 6), -7.0, np.float32)
    d2, c2 = np.full_like(d1, -9.0), np.full_like(c1, -9.0)
    for _ in range(3):  # frame 1 copies, frames 2-3 write straight into the mapped d1 / c1
        e.run_host(l, r, cloud=True, out=d1, cloud_out=c1)
        assert np.array_equal(d1, ref_d) and np.array_equal(c1, ref_c, equal_nan=True)
    d1[...] = -1.0
    c1[...] = -1.0
    for _ in range(2):  # swap: d2 / c2 receive the frames, d1 / c1 are left alone
        e.run_host(l, r, cloud=True, out=d2, cloud_out=c2)
        assert np.array_equal(d2, ref_d) and np.array_equal(c2, ref_c, equal_nan=True)
    assert (d1 == -1.0).all() and (c1 == -1.0).all()
    for _ in range(2):  # and back
        e.run_host(l, r, cloud=True, out=d1, cloud_out=c1)
        assert np.array_equal(d1, ref_d) and np.array_equal(c1, ref_c, equal_nan=True)
    # disparity only (no cloud requested): the disparity still lands in the caller's array
    d3 = np.zeros_like(d1)
    for _ in range(2):
        e.run_host(l, r, cloud=False, out=d3)
        assert np.array_equal(d3, ref_d)
    e.close()


def test_caller_inputs_zero_copy_and_fresh_arrays():
    """Zero-copy INPUTS (the frame graph's first node reads the caller's mapped arrays over PCIe): the same arrays
    refilled every frame (a camera's frame buffers) and fresh arrays every frame (a freed array's address comes back
    with other pages: the mapping must follow them) give, frame by frame, the pinned-I/O path's bytes for that
    frame's images -- outputs included."""
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    e = NativeStereoEngine("raftstereo-realtime", None, 480, 640, batch=1, device=0)
    e.set_Q(Q)
    pairs = [batch_pairs(1, 480, 640, seed=s) for s in (3, 4)]
    hb = e.host_buffers()
    refs = []
    for l, r in pairs:
        hb["left"][...] = l
        hb["right"][...] = r
        e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
        refs.append((hb["disp"].copy(), hb["cloud"].copy()))
    hb = None
    assert not np.array_equal(refs[0][0], refs[1][0])
    L, R = np.empty_like(pairs[0][0]), np.empty_like(pairs[0][1])
    d, c = np.empty((1, 480, 640), np.float32), np.empty((1, 480, 640, 6), np.float32)
    for k in range(5):  # mapped from the second frame on, new content every frame
        i = k % 2
        L[...] = pairs[i][0]
        R[...] = pairs[i][1]
        e.run_host(L, R, cloud=True, out=d, cloud_out=c)
        assert np.array_equal(d, refs[i][0]) and np.array_equal(c, refs[i][1], equal_nan=True), k
    del L, R, d, c
    for k in range(6):
        i = k % 2
        L, R = pairs[i][0].copy(), pairs[i][1].copy()
        d, c = np.empty((1, 480, 640), np.float32), np.empty((1, 480, 640, 6), np.float32)
        e.run_host(L, R, cloud=True, out=d, cloud_out=c)
        assert np.array_equal(d, refs[i][0]) and np.array_equal(c, refs[i][1], equal_nan=True), k
        del L, R, d, c
    e.close()


def test_run_device_writes_caller_tensors_from_the_graph():
    """the device run() path launches the frame graph with its input-copy node reading the caller's
    device images and its reprojection node writing disparity + cloud into the caller's tensors (no D2D copies around
    the graph).  Swapping out / cloud_out tensors between frames re-points the nodes: every frame's bytes equal the
    pinned-I/O run_host frame of the same images, a tensor no longer passed is not written, and changing the input
    tensors is followed frame by frame."""
    from stereoalgorithms_amd.models.engine import NativeStereoEngine
    b, h, w = 2, 240, 320
    e = NativeStereoEngine("raftstereo-realtime", None, h, w, batch=b, device=0)
    e.set_Q(Q)
    pairs = [batch_pairs(b, h, w, seed=s) for s in (3, 4)]
    refs = []
    hb = e.host_buffers()
    for l, r in pairs:
        hb["left"][...] = l
        hb["right"][...] = r
        e.run_host(hb["left"], hb["right"], cloud=True, out=hb["disp"], cloud_out=hb["cloud"])
        refs.append((torch.from_numpy(hb["disp"].copy()), torch.from_numpy(hb["cloud"].copy())))
    hb = None
    dev_pairs = [(torch.from_numpy(l).cuda(), torch.from_numpy(r).cuda()) for l, r in pairs]
    outs = [torch.full((b, h, w), -7.0, device="cuda") for _ in range(2)]
    clouds = [torch.full((b, h, w, 6), -7.0, device="cuda") for _ in range(2)]
    for i in range(6):
        k, j = i % 2, (i // 2) % 2  # output tensors alternate every frame, the input pair every two
        if i == 4:
            outs[1].fill_(-1.0)
            clouds[1].fill_(-1.0)
        l, r = dev_pairs[j]
        d, c = e.run(l, r, cloud=True, out=outs[k if i < 4 else 0], cloud_out=clouds[k if i < 4 else 0])
        torch.cuda.synchronize()
        assert torch.equal(d.cpu(), refs[j][0]), f"frame {i}: disparity"
        c_cpu, cref = c.cpu(), refs[j][1]
        assert torch.equal(torch.nan_to_num(c_cpu, 1e30), torch.nan_to_num(cref, 1e30)), f"frame {i}: cloud"
    assert (outs[1] == -1.0).all() and (clouds[1] == -1.0).all()  # frames 4-5 used only tensor 0
    d_only = torch.zeros(b, h, w, device="cuda")
    e.run(*dev_pairs[0], out=d_only)  # disparity only: still written by the graph
    torch.cuda.synchronize()
    assert torch.equal(d_only.cpu(), refs[0][0])
    e.close()
