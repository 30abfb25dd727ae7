"""Detection kernels + YOLOv8 on MI355X vs plain PyTorch fp32 references (BASELINE config 4)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_upsample2x_into_slice(native):
    from aiko_services_amd.ops import detect as DT
    x = torch.randn(2, 5, 7, 48, device=DEV).to(torch.bfloat16)
    big = torch.zeros(2, 10, 14, 80, dtype=torch.bfloat16, device=DEV)
    DT.upsample2x(x[..., 16:48], out=big[..., 48:80])
    ref = torch.nn.functional.interpolate(x[..., 16:48].permute(0, 3, 1, 2).float(), scale_factor=2,
                                          mode="nearest").permute(0, 2, 3, 1)
    assert torch.equal(big[..., 48:].float(), ref)
    assert big[..., :48].abs().max().item() == 0


def test_upsample2x_more_rows_than_grid_y(native):
    """B*H = 81920 image rows > 65535: the kernel strides over grid y."""
    from aiko_services_amd.ops import detect as DT
    x = torch.randn(2048, 40, 4, 8, device=DEV).to(torch.bfloat16)
    out = DT.upsample2x(x)
    ref = x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)
    assert torch.equal(out, ref)


def test_maxpool_slices(native):
    from aiko_services_amd.ops import vision as V
    cat = torch.randn(3, 20, 20, 128, device=DEV).to(torch.bfloat16)
    V.maxpool2d(cat[..., :32], 5, 1, 2, out=cat[..., 32:64])
    ref = torch.nn.functional.max_pool2d(cat[..., :32].permute(0, 3, 1, 2).float(), 5, 1, 2)
    assert torch.equal(cat[..., 32:64].permute(0, 3, 1, 2).float(), ref)


@pytest.mark.parametrize("cout", [16, 32, 144])
def test_conv_narrow_tiles_and_post_act_residual(native, cout):
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(cout)
    x = torch.randn(2, 40, 40, 48, generator=g).to(DEV, torch.bfloat16)
    w = torch.randn(cout, 32, 3, 3, generator=g) / 17
    b = torch.randn(cout, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, pad=1, act="silu", device=DEV)
    res = torch.randn(2, 40, 40, cout, generator=g).to(DEV, torch.bfloat16)
    ref = R.conv_ref(x[..., 8:40].permute(0, 3, 1, 2).float(), spec, res.permute(0, 3, 1, 2).float(),
                     residual_after_act=True)
    tiles = [(128, 32), (256, 32), (64, 64)] if cout <= 32 else [(128, 64), (64, 128)]
    for t in tiles:
        y = C.conv2d(x[..., 8:40], spec, residual=res, residual_after_act=True, tile=t)
        assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2, t


def test_letterbox_stem(native):
    from aiko_services_amd.models.yolov8 import YOLOv8
    from aiko_services_amd.ops import reference as R
    m = YOLOv8("n", device=DEV)
    frames = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8, device=DEV)
    pre = m.preprocess(frames)
    Ho, Wo, top, left, gain = m.letterbox((480, 640))
    assert (Ho, Wo, top, left) == (480, 640, 80, 0)
    canvas = torch.full((2, 3, 640, 640), 114.0 / 255, device=DEV)
    canvas[:, :, top:top + Ho, left:left + Wo] = frames.permute(0, 3, 1, 2).float() / 255
    assert _rel_err(pre[:, 1:641, 1:641, :3].permute(0, 3, 1, 2), canvas) < 5e-3
    assert pre[:, 0].abs().max().item() == 0 and pre[:, :, 0].abs().max().item() == 0
    y = torch.ops.aiko  # noqa: F841
    from aiko_services_amd.ops import conv as C
    a0 = C.conv2d(pre, m.l0, image_hw=(640, 640))
    ref = R.conv_ref(canvas.to(torch.bfloat16).float(), m.l0)
    assert a0.shape == (2, 320, 320, 16)
    assert _rel_err(a0.permute(0, 3, 1, 2), ref) < 1e-2


def test_yolo_decode(native):
    from aiko_services_amd.ops import detect as DT
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(5)
    feats = [(torch.randn(2, s, s, 144, generator=g) * 2).to(DEV, torch.bfloat16) for s in (16, 8, 4)]
    boxes, scores, cls = DT.yolo_decode(feats, (8, 16, 32), 80)
    rb, rs, rc = R.yolo_decode_ref([f.permute(0, 3, 1, 2) for f in feats], (8, 16, 32), 80)
    assert torch.allclose(boxes, rb, atol=1e-2, rtol=1e-4)
    assert torch.allclose(scores, rs, atol=1e-5)
    assert (cls == rc).float().mean().item() > 0.999


def test_yolo_decode_tiled_matches_per_anchor(native, monkeypatch):
    """The LDS-tiled decode and the per-anchor kernel (AIKO_DECODE_FLAT=1) give bit-identical
    boxes / scores / classes, incl. a partial last tile (5x5 = 25 anchors) and exact ties among
    class logits."""
    from aiko_services_amd.ops import detect as DT
    g = torch.Generator().manual_seed(9)
    feats = [(torch.randn(3, s, s, 144, generator=g) * 3).round().to(torch.bfloat16).to(DEV)
             for s in (20, 10, 5)]
    tiled = DT.yolo_decode(feats, (8, 16, 32), 80)
    monkeypatch.setenv("AIKO_DECODE_FLAT", "1")
    flat = DT.yolo_decode(feats, (8, 16, 32), 80)
    torch.cuda.synchronize()
    for a, b in zip(tiled, flat):
        assert torch.equal(a, b)


def _random_dets(B, A, g, n_centers=40, n_cls=3):
    centers = torch.rand(B, n_centers, 2, generator=g) * 600
    pick = torch.randint(0, n_centers, (B, A), generator=g)
    c = torch.gather(centers, 1, pick[..., None].expand(B, A, 2)) + torch.randn(B, A, 2, generator=g) * 6
    wh = 20 + torch.rand(B, A, 2, generator=g) * 60
    boxes = torch.cat([c - wh / 2, c + wh / 2], -1)
    scores = (torch.rand(B, A, generator=g) * 256).floor() / 256      # many exact ties
    cls = torch.randint(0, n_cls, (B, A), generator=g, dtype=torch.int32)
    return boxes.to(DEV), scores.to(DEV), cls.to(DEV)


# n_cls: 3 (class runs spanning several 64-candidate blocks), 1 (every block pair: the whole
# triangle), 80 (YOLO: mostly diagonal blocks), 1000 (a run per candidate); iou < 0: every pair
# suppresses, across classes too (one run in rank order)
@pytest.mark.parametrize("A,conf,max_cand,max_det,n_cls,iou", [
    (8400, 0.25, 1024, 300, 3, 0.5), (8400, 0.97, 1024, 300, 3, 0.5), (2000, 0.1, 256, 50, 3, 0.5),
    (33, 0.0, 1024, 300, 3, 0.5), (8400, 0.25, 1024, 300, 1, 0.5), (8400, 0.25, 1024, 1024, 1, 0.3),
    (8400, 0.25, 1024, 300, 80, 0.5), (8400, 0.25, 1000, 100, 1000, 0.5), (700, 0.1, 1024, 300, 80, -1.0),
    (6000, 0.5, 777, 13, 7, 0.45)])
def test_topk_nms_matches_reference(native, A, conf, max_cand, max_det, n_cls, iou):
    from aiko_services_amd.ops import detect as DT
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(A + max_det + n_cls)
    B = 3
    boxes, scores, cls = _random_dets(B, A, g, n_cls=n_cls)
    det, count = DT.topk_nms(boxes, scores, cls, conf=conf, iou=iou, max_candidates=max_cand,
                             max_det=max_det)
    torch.cuda.synchronize()
    for b in range(B):
        keep = R.nms_ref(boxes[b], scores[b], cls[b], conf, iou, max_cand, max_det)
        n = int(count[b])
        assert n == keep.numel(), (b, n, keep.numel())
        ref = torch.cat([boxes[b][keep].clamp(min=0), scores[b][keep, None], cls[b][keep, None].float()], 1)
        assert torch.allclose(det[b, :n], ref, atol=1e-4), b
        assert (det[b, n:, 5] == -1).all()


@pytest.mark.parametrize("hw", [(480, 640), (360, 500), (720, 1280)])
def test_stem_direct_matches_unfused(native, hw):
    """stem_direct_kernel (letterbox + /255 in LDS, direct 3x3/2 conv, bias, SiLU) equals
    preprocess + MFMA stem conv (resize and letterbox bars included)."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    m = YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(hw[0])
    frames = torch.randint(0, 256, (3,) + hw + (3,), generator=g, dtype=torch.uint8).to(DEV)
    fused = m.stem_from_frames(frames).clone()
    pre = m.preprocess(frames)
    unfused = C.conv2d(pre, m.l0, image_hw=(640, 640))
    assert fused.shape == unfused.shape == (3, 320, 320, 16)
    assert _rel_err(fused.float(), unfused.float()) < 5e-3
    canvas = pre[:, 1:641, 1:641, :3].permute(0, 3, 1, 2).float()
    ref = R.conv_ref(canvas, m.l0)
    assert _rel_err(fused.permute(0, 3, 1, 2), ref) < 1e-2


def test_fast_stem_wide_stores_identical(native, monkeypatch):
    """The fast stem's opt-in 16-B store path (v_permlane16_swap of the two half-row tiles)
    writes exactly the bytes of the 8-B store path, letterbox bars and ragged edges included."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(7)
    frames = torch.randint(0, 256, (2, 480, 640, 3), generator=g, dtype=torch.uint8).to(DEV)
    monkeypatch.setenv("AIKO_STEM_FAST_WIDE", "0")
    monkeypatch.setenv("AIKO_STEM_FAST_TH", "8")
    narrow = m.stem_from_frames(frames).clone()
    monkeypatch.setenv("AIKO_STEM_FAST_WIDE", "1")              # (8-row tiles only)
    wide = m.stem_from_frames(frames).clone()
    monkeypatch.setenv("AIKO_STEM_FAST_WIDE", "0")
    talls = []
    for th, tw in (("16", "32"), ("32", "32"), ("8", "64"), ("16", "64")):   # other tiles: same values
        monkeypatch.setenv("AIKO_STEM_FAST_TH", th)
        monkeypatch.setenv("AIKO_STEM_FAST_TW", tw)
        talls.append(m.stem_from_frames(frames).clone())
    torch.cuda.synchronize()
    assert torch.equal(wide, narrow)
    for tall in talls:
        assert torch.equal(tall, narrow)


def test_yolov8n_fused_stem_detect_matches(native):
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    frames = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8, device=DEV)
    a = [o.clone() for o in m.head_outputs(None, a0=m.stem_from_frames(frames))]
    b = m.head_outputs(m.preprocess(frames))
    for x, y in zip(a, b):
        cos = torch.nn.functional.cosine_similarity(x.float().flatten(), y.float().flatten(), dim=0).item()
        assert cos > 0.999, cos


def test_yolov8n_heads_match_reference(native):
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    frames = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8, device=DEV)
    outs = m.head_outputs(m.preprocess(frames))
    refs = m.reference_head_outputs(frames)
    for o, r in zip(outs, refs):
        o = o.permute(0, 3, 1, 2).float()
        cos = torch.nn.functional.cosine_similarity(o.flatten(), r.flatten(), dim=0).item()
        assert cos > 0.99, cos


def test_yolov8n_detect_end_to_end(native):
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    frames = torch.randint(0, 256, (4, 480, 640, 3), dtype=torch.uint8, device=DEV)
    det, count = m.detect(frames)
    torch.cuda.synchronize()
    assert det.shape == (4, 300, 6) and count.shape == (4,)
    for b in range(4):
        n = int(count[b])
        assert 0 <= n <= 300
        d = det[b, :n]
        if n:
            assert (d[:, 4] > 0.25).all() and (d[:, 4][:-1] >= d[:, 4][1:]).all()
            assert (d[:, 0] >= 0).all() and (d[:, 2] <= 640).all() and (d[:, 3] <= 480).all()


def test_example_yolo_element_overlay(native):
    """Reference-compatible YoloDetector (examples/yolo): list of numpy images -> overlay dict."""
    import queue

    import numpy as np

    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    d = {"version": 0, "name": "p_yolo_example", "runtime": "python", "graph": ["(YoloDetector)"],
         "parameters": {}, "elements": [
             {"name": "YoloDetector", "input": [{"name": "images", "type": "[image]"}],
              "output": [{"name": "overlay", "type": "[overlay]"}], "parameters": {"class_filter": "all"},
              "deploy": {"local": {"module": "aiko_services_amd.examples.yolo.yolo"}}}]}
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(d), None, None, "s", [], 0, None, 60,
                                     queue_response=q)
    rng = np.random.default_rng(0)
    images = [rng.integers(0, 256, (480, 640, 3), dtype=np.uint8) for _ in range(3)] + \
             [rng.integers(0, 256, (240, 320, 3), dtype=np.uint8)]
    p.process_frame({"stream_id": "s", "frame_id": 0}, {"images": images})
    info, out = q.get(timeout=60)
    assert info["state"] == 0, out
    ov = out["overlay"]
    assert len(ov["objects"]) == len(ov["rectangles"])
    for r in ov["rectangles"]:
        assert r["w"] >= 0 and r["h"] >= 0 and 0 <= r["x"] <= 640


def test_yolo_weights_roundtrip_bit_exact(native, tmp_path):
    """save() on one seed, load() into another: identical detections (packed weights + the
    re-derived fused head convs)."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    a = YOLOv8(scale="n", seed=0, device=DEV, image_size=320)
    b = YOLOv8(scale="n", seed=7, device=DEV, image_size=320)
    path = str(tmp_path / "yolo.safetensors")
    a.save(path)
    frames = torch.randint(0, 256, (2, 240, 320, 3), dtype=torch.uint8, device=DEV)
    det_a, cnt_a = (t.clone() for t in a.detect(frames))
    b.load(path)
    det_b, cnt_b = b.detect(frames)
    assert torch.equal(cnt_a, cnt_b) and torch.equal(det_a, det_b)


@pytest.mark.parametrize("rb", [10, 20, 160])
def test_c2f_fused_matches_unfused(native, monkeypatch, rb):
    """The one-launch C2f row stream (c2f_fused.hip) against the four-launch chain (cv1, bottleneck
    3x3 pair with the shortcut, cv2) on YOLOv8-n's l2 block: bands of rb rows (zero rows at the
    image edges, halo rows recomputed at band edges), two images."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(rb)
    x = (torch.randn(2, 160, 160, 32, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(YOLOv8, "_c2f_rb", staticmethod(lambda H: rb))
    out_f = torch.full((2, 160, 160, 32), 7.0, dtype=torch.bfloat16, device=DEV)
    assert m._c2f_fused_ok(m.l2, x, out_f)
    m._run_c2f("l2f", m.l2, x, out_f)
    monkeypatch.setenv("AIKO_C2F_FUSED", "0")
    out_u = torch.empty_like(out_f)
    m._run_c2f("l2u", m.l2, x, out_u)
    torch.cuda.synchronize()
    a, b = out_f.float(), out_u.float()
    cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    assert cos > 0.9995, cos
    assert (a - b).abs().max().item() < 0.05 * b.abs().max().item()


@pytest.mark.parametrize("rb", [10, 20, 80])
def test_c2f_fused_wide_matches_unfused(native, monkeypatch, rb):
    """The LDS-weights variant (c2f_fused_wl_kernel) on YOLOv8-n's l15 block (80 x 80, cv1 192 -> 64,
    bottleneck 3x3 32 -> 32 without the shortcut, cv2 96 -> 64) against the four-launch chain."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(rb)
    x = (torch.randn(2, 80, 80, 192, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(YOLOv8, "_c2f_rb", staticmethod(lambda H: rb))
    out_f = torch.full((2, 80, 80, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    assert m._c2f_fused_ok(m.l15, x, out_f)
    m._run_c2f("l15f", m.l15, x, out_f)
    monkeypatch.setenv("AIKO_C2F_FUSED", "0")
    out_u = torch.empty_like(out_f)
    m._run_c2f("l15u", m.l15, x, out_u)
    torch.cuda.synchronize()
    a, b = out_f.float(), out_u.float()
    cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    assert cos > 0.9995, cos
    assert (a - b).abs().max().item() < 0.05 * b.abs().max().item()


@pytest.mark.parametrize("rb", [10, 20])
def test_c2f_bneck_fused_matches_unfused(native, monkeypatch, rb):
    """The fused bottleneck pair (c2f_bneck_kernel) inside YOLOv8-n's l4 C2f (80 x 80, n = 2, the
    bottlenecks read / write channel slices of the concat buffer) against the unfused chain."""
    from aiko_services_amd.models.yolov8 import YOLOv8
    m = YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(rb)
    x = (torch.randn(2, 80, 80, 64, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(YOLOv8, "_c2f_rb", staticmethod(lambda H: rb))
    out_f = torch.empty(2, 80, 80, 64, dtype=torch.bfloat16, device=DEV)
    m._run_c2f("l4f", m.l4, x, out_f)
    monkeypatch.setenv("AIKO_C2F_FUSED", "0")
    out_u = torch.empty_like(out_f)
    m._run_c2f("l4u", m.l4, x, out_u)
    torch.cuda.synchronize()
    a, b = out_f.float(), out_u.float()
    cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    assert cos > 0.9995, cos
    assert (a - b).abs().max().item() < 0.05 * b.abs().max().item()


@pytest.mark.parametrize("hw", [(80, 80), (40, 40), (20, 20)])
def test_conv_tail_matches_two_convs(native, monkeypatch, hw):
    """Detect-head class branch as ONE launch (conv_glds TAIL: 3x3 80 -> 80 + SiLU with the 1x1
    80 -> 80 logits in the epilogue) against the two separate convs, at the three head levels;
    input and output are channel slices of the head's [.., 64 + 80] buffers."""
    from aiko_services_amd.models import yolov8 as Y
    from aiko_services_amd.ops import conv as C
    m = Y.YOLOv8("n", device=DEV)
    lvl = m.heads[0]
    g = torch.Generator().manual_seed(hw[0])
    h1 = (torch.randn(2, hw[0], hw[1], 144, generator=g) * 2).to(DEV, torch.bfloat16)
    out_f = torch.full((2, hw[0], hw[1], 144), 7.0, dtype=torch.bfloat16, device=DEV)
    assert C.conv_tail_ok(h1[..., 64:], lvl.cls[1], lvl.cls[2])
    C.conv2d_tail(h1[..., 64:], lvl.cls[1], lvl.cls[2], out_f[..., 64:])
    t = C.conv2d(h1[..., 64:], lvl.cls[1])
    ref = C.conv2d(t, lvl.cls[2])
    torch.cuda.synchronize()
    assert torch.equal(out_f[..., :64], torch.full_like(out_f[..., :64], 7.0))   # box slice untouched
    a, b = out_f[..., 64:].float(), ref.float()
    cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
    assert cos > 0.9999, cos
    assert (a - b).abs().max().item() < 0.02 * b.abs().max().item()
    # fp32 reference of the same two convs
    xr = h1[..., 64:].float().permute(0, 3, 1, 2)
    tr = torch.nn.functional.silu(torch.nn.functional.conv2d(xr, lvl.cls[1].ref_weight.to(DEV), lvl.cls[1].ref_bias.to(DEV), padding=1))
    yr = torch.nn.functional.conv2d(tr, lvl.cls[2].ref_weight.to(DEV), lvl.cls[2].ref_bias.to(DEV)).permute(0, 2, 3, 1)
    assert ((a - yr).norm() / yr.norm()).item() < 1e-2
    # the model's level-0 head with and without the fused class branch
    p3 = (torch.randn(2, hw[0], hw[1], 64, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(Y, "_HEAD_TAIL", True)
    o_f = m._run_head(0, lvl, p3).clone()
    monkeypatch.setattr(Y, "_HEAD_TAIL", False)
    o_u = m._run_head(0, lvl, p3).clone()
    torch.cuda.synchronize()
    for sl in (slice(0, 64), slice(64, 144)):              # box (64) and class (80) branches
        a, b = o_f[..., sl].float(), o_u[..., sl].float()
        assert torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item() > 0.9999
    # the box branch alone (64 -> 64 tail) against the fp32 reference
    bo = torch.full((2, hw[0], hw[1], 144), 7.0, dtype=torch.bfloat16, device=DEV)
    assert C.conv_tail_ok(h1[..., :64], lvl.box[1], lvl.box[2])
    C.conv2d_tail(h1[..., :64], lvl.box[1], lvl.box[2], bo[..., :64])
    torch.cuda.synchronize()
    assert torch.equal(bo[..., 64:], torch.full_like(bo[..., 64:], 7.0))
    xr = h1[..., :64].float().permute(0, 3, 1, 2)
    tr = torch.nn.functional.silu(torch.nn.functional.conv2d(xr, lvl.box[1].ref_weight.to(DEV), lvl.box[1].ref_bias.to(DEV), padding=1))
    yr = torch.nn.functional.conv2d(tr, lvl.box[2].ref_weight.to(DEV), lvl.box[2].ref_bias.to(DEV)).permute(0, 2, 3, 1)
    a = bo[..., :64].float()
    assert ((a - yr).norm() / yr.norm()).item() < 1e-2


def test_yolo_tails_match_unfused(native, monkeypatch):
    """The whole YOLOv8-n head_outputs with the fused 3x3 + 1x1 launches (l3 -> l4.cv1 with SiLU,
    detect-head box and class branches) against the same network with every conv separate."""
    from aiko_services_amd.models import yolov8 as Y
    m = Y.YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(11)
    a0 = (torch.randn(2, 320, 320, 16, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(Y, "_HEAD_TAIL", True)
    fused = [o.clone() for o in m.head_outputs(None, a0=a0)]
    monkeypatch.setattr(Y, "_HEAD_TAIL", False)
    plain = [o.clone() for o in m.head_outputs(None, a0=a0)]
    torch.cuda.synchronize()
    for a, b in zip(fused, plain):
        a, b = a.float(), b.float()
        cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
        assert cos > 0.999, cos


def test_yolo_upsample_inplace_matches(native, monkeypatch):
    """l15's fused C2f reading up(l12) in place from a12 (no upsample2x kernel, the upsampled half
    of its input buffer never written) gives bit-identical head outputs."""
    from aiko_services_amd.models import yolov8 as Y
    m = Y.YOLOv8("n", device=DEV)
    g = torch.Generator().manual_seed(12)
    a0 = (torch.randn(2, 320, 320, 16, generator=g) * 2).to(DEV, torch.bfloat16)
    monkeypatch.setattr(Y, "_UP_INPLACE", True)
    fused = [o.clone() for o in m.head_outputs(None, a0=a0)]
    monkeypatch.setattr(Y, "_UP_INPLACE", False)
    plain = [o.clone() for o in m.head_outputs(None, a0=a0)]
    torch.cuda.synchronize()
    for a, b in zip(fused, plain):
        assert torch.equal(a, b)


def test_yolo_decode_in_tail_matches_decode_kernel(native, monkeypatch):
    """The detect head's tail launches decoding in their epilogues (DFL -> xyxy boxes, sigmoid(max)
    / argmax) against the stored head outputs + the yolo_decode kernel, and the final detections."""
    from aiko_services_amd.models import yolov8 as Y
    from aiko_services_amd.ops import detect as DT
    m = Y.YOLOv8("n", device=DEV, cls_bias=0.0)
    assert m._decode_fused_ok()
    g = torch.Generator().manual_seed(13)
    a0 = (torch.randn(2, 320, 320, 16, generator=g) * 2).to(DEV, torch.bfloat16)
    bf, sf, cf = (t.clone() for t in m.head_outputs(None, a0=a0, decode=True))
    feats = m.head_outputs(None, a0=a0)
    A = sum(f.shape[1] * f.shape[2] for f in feats)
    bd, sd, cd = DT.yolo_decode(feats, Y.STRIDES, m.nc_pad, boxes=torch.empty(2, A, 4, device=DEV),
                                scores=torch.empty(2, A, device=DEV), cls=torch.empty(2, A, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    assert torch.equal(cf, cd)
    assert torch.equal(sf, sd)
    assert (bf - bd).abs().max().item() < 1e-3 * bd.abs().max().item()
    # whole detect(): fused decode vs the decode kernel (same front end for both)
    frames = torch.randint(0, 256, (2, 480, 640, 3), generator=g, dtype=torch.uint8).to(DEV)
    det_f, cnt_f = (t.clone() for t in m.detect(frames))
    monkeypatch.setattr(Y, "_DECODE_FUSED", False)
    det_d, cnt_d = (t.clone() for t in m.detect(frames))
    torch.cuda.synchronize()
    assert torch.equal(cnt_f, cnt_d)
    assert (det_f - det_d).abs().max().item() < 1e-2 * max(1.0, det_d.abs().max().item())


@pytest.mark.parametrize("B", [96, 160])
def test_topk_nms_workgroups_per_image(native, B):
    """The fused NMS splits each image over G = CUs / B workgroups (at most 4, last arriver runs
    the scan): B = 96 gives G = 2 on a 256-CU MI355X, B = 160 gives G = 1 (everything in LDS);
    B = 3 (test_topk_nms_matches_reference) gives G = 4.  Every image equals nms_ref."""
    from aiko_services_amd.ops import detect as DT
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B)
    boxes, scores, cls = _random_dets(B, 3000, g, n_cls=2)
    det, count = DT.topk_nms(boxes, scores, cls, conf=0.2, iou=0.5, max_candidates=1024, max_det=300)
    torch.cuda.synchronize()
    for b in range(0, B, 7):
        keep = R.nms_ref(boxes[b], scores[b], cls[b], 0.2, 0.5, 1024, 300)
        n = int(count[b])
        assert n == keep.numel(), (b, n, keep.numel())
        ref = torch.cat([boxes[b][keep].clamp(min=0), scores[b][keep, None], cls[b][keep, None].float()], 1)
        assert torch.allclose(det[b, :n], ref, atol=1e-4), b
