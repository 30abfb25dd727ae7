"""Numerical parity AT THE CREDITED BENCH SHAPES.

The tuner keys its tile picks on the layer geometry, so the bench batches — B = 640 (ResNet-50
headline) and B = 192 (YOLOv8-n, config 4), ``bench.parse_args`` defaults — run kernels (256 x 256 conv_wide, conv_wide_pers, patchw, chain2,
conv_pw_rb, the detect-head tail-decode launches) that the small-batch parity tests never reach.
These tests build the bench pipelines exactly as ``bench.py`` does (``bench.definition`` /
``bench.yolo_definition``: tuner picks, 2 frame lanes, hipGraph capture per pool slot and lane),
run the setup frames, then compare REPLAYED steps of both lanes against the fp32 PyTorch
references (``ResNet50.reference_logits``; ``YOLOv8.reference_head_outputs`` decoded by
``ops.reference.yolo_decode_ref`` + ``nms_ref``).  Each check is also run on a sabotaged model
(one stage-3 conv's packed kernel weights zeroed after capture, the fp32 reference weights
untouched — what a wrong tile or a broken kernel looks like from outside) and must FAIL there,
so the comparison has teeth.

Reference element served: /root/reference/src/aiko_services/examples/yolo/yolo.py:56-87;
headline pipeline: /root/reference/src/aiko_services/main/pipeline.py:1037-1092.
"""
import os
import queue
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _pipeline(d):
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<parity>", parse_pipeline_definition_dict(d), None, None, "par", [], 0,
                                     None, 600, queue_response=q)
    p.response_swag = True          # the whole swag (inputs and intermediate outputs) comes back
    return p, q


def _element(p, name):
    return p.pipeline_graph.get_node(name).element


def _run(p, q, frame_id, result_key):
    p.process_frame({"stream_id": "par", "frame_id": frame_id}, {})
    info, swag = q.get_nowait()
    assert info["state"] == 0, (info, swag)
    swag[result_key].wait()
    torch.cuda.synchronize()
    return swag


# ---- ResNet-50 at the bench batch, 2 lanes, hipGraph (BASELINE config 2, the credited headline) --
RESNET_SETUP = 12          # bench.SETUP_FRAMES: tune + one capture per pool slot (6) and lane (2)
CHECK_FRAMES = 16          # frames compared per replayed step


def _resnet_parity(sabotage: bool):
    import bench
    B = bench.parse_args([]).batch
    p, q = _pipeline(bench.definition(B, True, 224, 224, 2))
    for fid in range(RESNET_SETUP):
        _run(p, q, fid, "topk")
    model = _element(p, "ResNet50Classifier").model
    if sabotage:
        model.blocks[9].conv2.weight[:64].zero_()      # kernel weights only; ref_weight untouched
    results = []
    for fid in range(RESNET_SETUP, RESNET_SETUP + 2):  # one replayed step on each lane
        swag = _run(p, q, fid, "topk")
        images = swag["images"][:CHECK_FRAMES].clone()
        logits = swag["logits"][:CHECK_FRAMES].float().clone()
        top = swag["topk"].wait()["top_index"][:CHECK_FRAMES].long().cpu()
        ref = model.reference_logits(images).float()
        torch.cuda.synchronize()
        cos = torch.nn.functional.cosine_similarity(logits, ref, dim=1).cpu()
        r2 = ref.topk(2, dim=1).values.cpu()
        margin = r2[:, 0] - r2[:, 1]
        err = (logits - ref).abs().max(dim=1).values.cpu()
        decisive = margin > 2 * err                     # fp32 top-1 not within bf16 error of top-2
        agree = top[:, 0] == ref.argmax(1).cpu()
        results.append({"cos": cos, "decisive": decisive, "agree": agree, "lane": swag.get("lane")})
    return results


COS_MIN = 0.9999           # measured clean: > 0.99999 per frame (bf16 kernels vs fp32 reference)


def _resnet_ok(results):
    for r in results:
        if r["cos"].min().item() <= COS_MIN:
            return False
        if not bool(r["agree"][r["decisive"]].all()):
            return False
    return True


def test_resnet50_bench_shape_matches_fp32_reference(native):
    results = _resnet_parity(sabotage=False)
    print("resnet50 bench-batch parity: min cos", [round(r["cos"].min().item(), 7) for r in results])
    for r in results:
        assert r["cos"].min().item() > COS_MIN, r["cos"]
        assert bool(r["agree"][r["decisive"]].all()), (r["agree"], r["decisive"])
        assert int(r["decisive"].sum()) >= CHECK_FRAMES // 2, r["decisive"]


def test_resnet50_bench_shape_check_catches_a_wrong_kernel(native):
    results = _resnet_parity(sabotage=True)
    print("resnet50 sabotaged: min cos", [round(r["cos"].min().item(), 7) for r in results])
    assert not _resnet_ok(results)


# ---- YOLOv8-n at the bench batch, 480 x 640 frames, tail-decode head, 2 lanes, hipGraph (config 4)
# With random-init weights the detections are a dense band of near-tied scores (~0.3, many exact
# bf16 ties), so comparing two NMS outputs would test the conditioning of greedy NMS, not the
# kernels.  The parity is therefore split at the decode: (1) the tail launches' decoded rows
# (every anchor's box, max-class score and class, read from the lane's workspace after the
# replay) against the fp32 reference head decoded by ops.reference.yolo_decode_ref, and (2) the
# NMS kernel's detections against nms_ref run on those SAME decoded rows, exactly.
YOLO_SETUP = 8             # pool 4 x 2 lanes
SCORE_TOL = 0.03           # |sigmoid(max logit)| kernel (bf16 network) vs fp32
BOX_TOL = 2.0              # canvas pixels (DFL expectation; strides 8 / 16 / 32)


def _map_back(boxes, frame_hw, geom):
    Ho, Wo, top, left, gain = geom
    H, W = frame_hw
    out = boxes.clone()
    out[:, [0, 2]] = ((out[:, [0, 2]] - left) / gain).clamp(0, W)
    out[:, [1, 3]] = ((out[:, [1, 3]] - top) / gain).clamp(0, H)
    return out


def _yolo_parity(sabotage: bool):
    import bench
    from aiko_services_amd.ops import reference as R
    B = bench.parse_args(["--model", "yolov8n"]).batch
    p, q = _pipeline(bench.yolo_definition(B, True, 480, 640, "scatter", 2))
    for fid in range(YOLO_SETUP):
        _run(p, q, fid, "detections")
    m = _element(p, "YoloDetector").model
    if sabotage:
        m.heads[0].cls[2].weight[:40].zero_()            # level-0 class 1x1 (a tail launch): kernel weights only
    n_images = 8
    out = {"score_max": 0.0, "score_mean": 0.0, "box_max": 0.0, "cls_bad": 0, "cls_n": 0, "nms_exact": True,
           "dets": 0}
    for fid in range(YOLO_SETUP, YOLO_SETUP + 2):        # one replayed step on each lane
        swag = _run(p, q, fid, "detections")
        frames = swag["images"][:n_images].clone()
        res = swag["detections"].wait()
        det, count = res["det"][:n_images].clone(), res["count"][:n_images].clone()
        A = sum((640 // s) ** 2 for s in (8, 16, 32))
        feats = m.reference_head_outputs(frames)
        rb, rs, rc = R.yolo_decode_ref(feats, (8, 16, 32), m.nc)
        # the decoded rows stay in the workspace of the lane that ran the frame (the lane is not
        # visible once the frame left the pipeline): the lane whose rows are this frame's
        lanes = [t for t in ("", "lane1.") if (t + "scores", (B, A), torch.float32) in m._ws]
        tag = min(lanes, key=lambda t: (m._ws[(t + "scores", (B, A), torch.float32)][:n_images] - rs).abs().mean().item())
        kb = m._ws[(tag + "boxes", (B, A, 4), torch.float32)][:n_images].clone()
        ks = m._ws[(tag + "scores", (B, A), torch.float32)][:n_images].clone()
        kc = m._ws[(tag + "cls", (B, A), torch.int32)][:n_images].clone()
        torch.cuda.synchronize()
        # (1) decode parity over every anchor
        ds = (ks - rs).abs()
        out["score_max"] = max(out["score_max"], ds.max().item())
        out["score_mean"] = max(out["score_mean"], ds.mean().item())
        logits = torch.cat([f[:, 64:].reshape(n_images, m.nc, -1) for f in feats], 2)      # [B, nc, A]
        top2 = logits.topk(2, dim=1).values
        decisive = (top2[:, 0] - top2[:, 1]) > 0.1                                         # class margin
        out["cls_bad"] += int(((kc != rc) & decisive).sum())
        out["cls_n"] += int(decisive.sum())
        lit = rs > 0.1                                                                      # boxes that matter
        if lit.any():
            out["box_max"] = max(out["box_max"], (kb - rb).abs().amax(-1)[lit].max().item())
        # (2) NMS exact on the kernel's own decoded rows
        geom = m.letterbox(frames.shape[1:3])
        for b in range(n_images):
            keep = R.nms_ref(kb[b], ks[b], kc[b], m.conf, m.iou, m.max_candidates, m.max_det)
            ref = torch.cat([_map_back(kb[b][keep], frames.shape[1:3], geom), ks[b][keep, None],
                             kc[b][keep, None].float()], 1)
            n = int(count[b])
            out["dets"] += n
            if n != keep.numel() or not torch.allclose(det[b, :n].to(ref.device), ref, atol=1e-3):
                if out["nms_exact"]:
                    d = det[b, :n].to(ref.device)
                    k = min(n, keep.numel())
                    bad = (d[:k] - ref[:k]).abs().amax(1) > 1e-3
                    i = int(bad.nonzero()[0]) if bad.any() else k
                    print("nms mismatch image", b, "n", n, "ref", keep.numel(), "first row", i,
                          d[i:i + 2].tolist() if i < n else None, ref[i:i + 2].tolist() if i < keep.numel() else None,
                          "above conf", int((ks[b] > m.conf).sum()))
                out["nms_exact"] = False
    print("yolov8n bench-batch parity:", out)
    return out


def _yolo_ok(r):
    return (r["score_max"] < SCORE_TOL and r["box_max"] < BOX_TOL and r["cls_n"] > 1000
            and r["cls_bad"] <= 1e-3 * r["cls_n"] and r["nms_exact"] and r["dets"] > 0)


def test_yolov8n_bench_shape_matches_reference(native):
    assert _yolo_ok(_yolo_parity(sabotage=False))


def test_yolov8n_bench_shape_check_catches_a_wrong_kernel(native):
    assert not _yolo_ok(_yolo_parity(sabotage=True))
