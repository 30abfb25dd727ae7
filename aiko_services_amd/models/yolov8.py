"""YOLOv8 (n/s/m/l/x) detection on aiko_services_amd's HIP kernels — NHWC bf16, BN folded.

The reference runs Ultralytics YOLOv8 inside ``YoloDetector`` (``examples/yolo/yolo.py:46-87``,
SURVEY §2.4 K4); BASELINE config 4 is 8x data-parallel YOLOv8-n.  Here the network is built
only from our ops and executed as a fixed launch sequence (hipGraph-capturable):

  letterbox preprocess (u8 -> 640x640 canvas, fill 114, /255, zero-bordered 4-channel buffer)
  -> stem 3x3/2 igemm (Cc = 16 pixel-run trick) -> backbone convs / C2f / SPPF
  -> PAN neck (upsample2x and conv outputs written straight into concat-buffer channel slices:
     no concat copies) -> decoupled Detect head (box|cls first convs fused along Cout)
  -> DFL decode kernel -> fused top-k + class-aware NMS kernel -> [B, max_det, 6] + counts.

C2f blocks keep their split/concat in ONE buffer [B, H, W, (2+n)c]: cv1 writes channels
[0, 2c), bottleneck i reads slice [(1+i)c, (2+i)c) and writes [(2+i)c, (3+i)c) with the
``x + silu(conv(x))`` shortcut done in the igemm epilogue (residual-after-activation), cv2
reads the whole buffer.  SPPF's cascaded 5x5 max-pools write slices of its concat buffer.

Weights are random-init (no checkpoints offline; the reference's ``yolov8n_robotdog.pt`` is
absent), deterministic per seed, BatchNorm folded at construction.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from ..ops import conv as C
from .weights import WeightsMixin
from ..ops import detect as DT
from ..ops import vision as V

# scale: (depth multiple, width multiple, max channels) as in the YOLOv8 model family
SCALES = {"n": (0.33, 0.25, 1024), "s": (0.33, 0.50, 1024), "m": (0.67, 0.75, 768),
          "l": (1.00, 1.00, 512), "x": (1.00, 1.25, 512)}
STRIDES = (8, 16, 32)
REG_MAX = 16
# the detect head's class branch as one conv_glds launch with the 1x1 in its epilogue
# (AIKO_HEAD_TAIL=0: the two separate convs)
_HEAD_TAIL = __import__("os").environ.get("AIKO_HEAD_TAIL", "1") != "0"
# (and the box branch, 3x3 64 -> 64 + 1x1 64 -> 64, the same way)
# the detect head's tail launches decode in their epilogues (AIKO_DECODE_FUSED=0: head outputs +
# the yolo_decode kernel)
_DECODE_FUSED = __import__("os").environ.get("AIKO_DECODE_FUSED", "1") != "0"
# l15's fused C2f reads the 2x upsample of l12 in place (+1.6 % over 5 interleaved bench pairs
# against the upsample2x kernel, round 5)
_UP_INPLACE = True


def _make_div(x, d=8):
    return int(math.ceil(x / d) * d)


def _rand_bn(g, c):
    gamma = 0.5 + 0.5 * torch.rand(c, generator=g)
    beta = 0.1 * torch.randn(c, generator=g)
    mean = 0.1 * torch.randn(c, generator=g)
    var = 0.5 + torch.rand(c, generator=g)
    return gamma, beta, mean, var


def _conv_bn(g, cin, cout, k, s=1, device=None, stem=False):
    """Conv2d(bias=False) + BatchNorm2d + SiLU (Ultralytics ``Conv``), folded and packed."""
    w = torch.randn(cout, cin, k, k, generator=g) * math.sqrt(2.0 / (cin * k * k))
    wf, b = C.fold_bn(w, *_rand_bn(g, cout))
    if stem:
        return C.make_stem_spec(wf, b, act="silu", device=device, stride=s, pad=k // 2)
    return C.make_conv_spec(wf, b, stride=s, pad=k // 2, act="silu", device=device)


def concat_cout(a: C.ConvSpec, b: C.ConvSpec) -> C.ConvSpec:
    """Two convs over the same input as ONE igemm with Cout = a.cout + b.cout."""
    assert (a.R, a.S, a.stride, a.pad, a.Cc, a.K, a.act) == (b.R, b.S, b.stride, b.pad, b.Cc, b.K, b.act)
    bias = torch.cat([a.bias, b.bias]) if a.bias is not None and b.bias is not None else None
    return C.ConvSpec(weight=torch.cat([a.weight, b.weight]).contiguous(), bias=bias, cin=a.cin,
                      cout=a.cout + b.cout, R=a.R, S=a.S, stride=a.stride, pad=a.pad, Cc=a.Cc,
                      act=a.act, kind="conv")


@dataclass
class C2f:
    cv1: C.ConvSpec
    cv2: C.ConvSpec
    m: list = field(default_factory=list)     # [(conv a, conv b)]
    c: int = 0
    shortcut: bool = True


@dataclass
class SPPF:
    cv1: C.ConvSpec
    cv2: C.ConvSpec
    k: int = 5


@dataclass
class DetectLevel:
    box: list          # 3 specs: 3x3, 3x3, 1x1(no act)
    cls: list
    first: C.ConvSpec  # box[0] | cls[0] fused along Cout


class YOLOv8(WeightsMixin):
    """Packed YOLOv8 detector.  ``detect(frames_u8) -> (det [B, max_det, 6], count [B])``."""

    def __init__(self, scale: str = "n", num_classes: int = 80, seed: int = 0, device="cuda",
                 image_size: int = 640, cls_bias: float = -2.4, conf: float = 0.25,
                 iou: float = 0.7, max_det: int = 300, max_candidates: int = 1024):
        self.device = torch.device(device)
        self.scale = scale
        self.nc = num_classes
        self.image_size = image_size
        self.conf, self.iou, self.max_det, self.max_candidates = conf, iou, max_det, max_candidates
        # the class conv's Cout is padded to a multiple of 8 (16-byte epilogue chunks); padded
        # classes have zero weights and a -40 logit bias, so they never pass any threshold
        self.nc_pad = -(-num_classes // 8) * 8
        d, w, mc = SCALES[scale]
        ch = lambda x: _make_div(min(x, mc) * w)  # noqa: E731
        rep = lambda n: max(round(n * d), 1)        # noqa: E731
        c1, c2, c3, c4, c5 = ch(64), ch(128), ch(256), ch(512), ch(1024)
        self.ch = (c1, c2, c3, c4, c5)
        g = torch.Generator().manual_seed(seed)
        dev = self.device
        self.l0 = _conv_bn(g, 3, c1, 3, 2, dev, stem=True)
        self.l1 = _conv_bn(g, c1, c2, 3, 2, dev)
        self.l2 = self._c2f(g, c2, c2, rep(3), True)
        self.l3 = _conv_bn(g, c2, c3, 3, 2, dev)
        self.l4 = self._c2f(g, c3, c3, rep(6), True)
        self.l5 = _conv_bn(g, c3, c4, 3, 2, dev)
        self.l6 = self._c2f(g, c4, c4, rep(6), True)
        self.l7 = _conv_bn(g, c4, c5, 3, 2, dev)
        self.l8 = self._c2f(g, c5, c5, rep(3), True)
        self.l9 = SPPF(_conv_bn(g, c5, c5 // 2, 1, 1, dev), _conv_bn(g, c5 // 2 * 4, c5, 1, 1, dev))
        self.l12 = self._c2f(g, c5 + c4, c4, rep(3), False)
        self.l15 = self._c2f(g, c4 + c3, c3, rep(3), False)
        self.l16 = _conv_bn(g, c3, c3, 3, 2, dev)
        self.l18 = self._c2f(g, c3 + c4, c4, rep(3), False)
        self.l19 = _conv_bn(g, c4, c4, 3, 2, dev)
        self.l21 = self._c2f(g, c4 + c5, c5, rep(3), False)
        cb = max(16, c3 // 4, REG_MAX * 4)
        cc = max(c3, min(num_classes, 100))
        self.cb, self.cc = cb, cc
        self.heads = []
        for i, cin in enumerate((c3, c4, c5)):
            box = [_conv_bn(g, cin, cb, 3, 1, dev), _conv_bn(g, cb, cb, 3, 1, dev)]
            wbox = 1.0 * torch.randn(4 * REG_MAX, cb, 1, 1, generator=g)
            box.append(C.make_conv_spec(wbox, torch.ones(4 * REG_MAX), act=None, device=dev))
            cls = [_conv_bn(g, cin, cc, 3, 1, dev), _conv_bn(g, cc, cc, 3, 1, dev)]
            wcls = torch.zeros(self.nc_pad, cc, 1, 1)
            wcls[:num_classes] = 0.9 * torch.randn(num_classes, cc, 1, 1, generator=g)
            bcls = torch.full((self.nc_pad,), -40.0)
            bcls[:num_classes] = float(cls_bias)
            cls.append(C.make_conv_spec(wcls, bcls, act=None, device=dev))
            self.heads.append(DetectLevel(box, cls, concat_cout(box[0], cls[0])))
        self._ws: dict = {}
        self.fused_stem = True            # stem_direct_kernel (letterbox + stem conv fused)
        self._stem_w = None
        self.ws_tag = ""             # workspace key prefix (one workspace per frame lane)

    def _c2f(self, g, cin, cout, n, shortcut):
        c = cout // 2
        dev = self.device
        cv1 = _conv_bn(g, cin, 2 * c, 1, 1, dev)
        cv2 = _conv_bn(g, (2 + n) * c, cout, 1, 1, dev)
        m = [(_conv_bn(g, c, c, 3, 1, dev), _conv_bn(g, c, c, 3, 1, dev)) for _ in range(n)]
        return C2f(cv1, cv2, m, c, shortcut)

    # ---- workspace ----------------------------------------------------------------------------
    def _buf(self, key, shape, dtype=torch.bfloat16):
        k = (self.ws_tag + key, tuple(shape), dtype)
        t = self._ws.get(k)
        if t is None:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._ws[k] = t
        return t

    def release_workspace(self):
        self._ws.clear()

    # ---- blocks -------------------------------------------------------------------------------
    def _c2f_fused_ok(self, blk: C2f, x, out) -> bool:
        """The one-launch C2f row stream (``c2f_fused.hip``) has this shape: one bottleneck, 160-wide
        rows, 32 -> (16 | 16) -> 32 channels with the shortcut (YOLOv8-n l2)."""
        import os
        if not x.is_cuda or os.environ.get("AIKO_C2F_FUSED", "1") == "0" or len(blk.m) != 1:
            return False
        a, b = blk.m[0]
        B, H, W, _ = x.shape
        shape = (W, blk.cv1.Cc, blk.c, blk.cv2.cout, blk.shortcut)
        return (shape in ((160, 32, 16, 32, True), (80, 192, 32, 64, False)) and H % self._c2f_rb(H) == 0
                and a.R == 3 and b.R == 3 and a.Cc == blk.c and b.Cc == blk.c
                and x.stride(3) == 1 and out.stride(3) == 1)

    @staticmethod
    def _c2f_rb(H):
        """Band height: 160-row images 40 (bench sweep 32-160), 80-row images 20."""
        return 40 if H == 160 else 20

    def _run_c2f(self, name, blk: C2f, x, out, cat=None, xu=None):
        """``cat``: the block's split/concat buffer with cv1's output already in channels
        [0, 2c) (``x`` then only gives the shape).  ``xu``: the fused kernel reads x's first
        ``xu.shape[3]`` channels as the nearest 2x upsample of ``xu`` (only with the fused C2f)."""
        B, H, W, _ = x.shape
        c, n = blk.c, len(blk.m)
        if cat is None and self._c2f_fused_ok(blk, x, out):
            a, b = blk.m[0]
            torch.ops.aiko.c2f_fused_out(x, blk.cv1.weight, blk.cv1.bias, a.weight, a.bias, b.weight, b.bias,
                                         blk.cv2.weight, blk.cv2.bias, out, blk.cv1.Cc, blk.shortcut, self._c2f_rb(H),
                                         xu)
            return out
        if xu is not None:
            raise ValueError("_run_c2f: an in-place upsample source needs the fused C2f kernel")
        if cat is None:
            cat = self._buf(f"{name}.cat", (B, H, W, (2 + n) * c))
            C.conv2d(x, blk.cv1, out=cat[..., :2 * c])
        tmp = self._buf(f"{name}.tmp", (B, H, W, c))
        import os
        fuse_b = (cat.is_cuda and os.environ.get("AIKO_C2F_FUSED", "1") != "0" and W == 80 and c == 32
                  and blk.shortcut and H % self._c2f_rb(H) == 0)
        for i, (a, b) in enumerate(blk.m):
            src = cat[..., (1 + i) * c:(2 + i) * c]
            if fuse_b and a.R == 3 and b.R == 3 and a.Cc == c and b.Cc == c:
                # both 3x3 convs + shortcut in one row-stream launch (t stays in LDS)
                torch.ops.aiko.c2f_bneck_out(src, a.weight, a.bias, b.weight, b.bias,
                                             cat[..., (2 + i) * c:(3 + i) * c], blk.shortcut, self._c2f_rb(H))
                continue
            C.conv2d(src, a, out=tmp)
            C.conv2d(tmp, b, out=cat[..., (2 + i) * c:(3 + i) * c],
                     residual=src if blk.shortcut else None, residual_after_act=True)
        C.conv2d(cat, blk.cv2, out=out)
        return out

    def _run_sppf(self, name, blk: SPPF, x, out):
        B, H, W, _ = x.shape
        c = blk.cv1.cout
        cat = self._buf(f"{name}.cat", (B, H, W, 4 * c))
        C.conv2d(x, blk.cv1, out=cat[..., :c])
        if cat.is_cuda and H * W <= 2048 and c % 8 == 0:
            V.sppf_pool(cat, c, blk.k)          # the three chained pools in one kernel
            return C.conv2d(cat, blk.cv2, out=out)
        for i in range(3):
            V.maxpool2d(cat[..., i * c:(i + 1) * c], blk.k, 1, blk.k // 2, out=cat[..., (i + 1) * c:(i + 2) * c])
        C.conv2d(cat, blk.cv2, out=out)
        return out

    def _run_head(self, i, lvl: DetectLevel, x):
        B, H, W, _ = x.shape
        cb, cc = self.cb, self.cc
        h1 = self._buf(f"h{i}.1", (B, H, W, cb + cc))
        h2 = self._buf(f"h{i}.2", (B, H, W, cb + cc))
        out = self._buf(f"h{i}.out", (B, H, W, 4 * REG_MAX + self.nc_pad))
        C.conv2d(x, lvl.first, out=h1)
        if _HEAD_TAIL and C.conv_tail_ok(h1[..., :cb], lvl.box[1], lvl.box[2]):
            C.conv2d_tail(h1[..., :cb], lvl.box[1], lvl.box[2], out[..., :4 * REG_MAX])
        else:
            C.conv2d(h1[..., :cb], lvl.box[1], out=h2[..., :cb])
            C.conv2d(h2[..., :cb], lvl.box[2], out=out[..., :4 * REG_MAX])
        if _HEAD_TAIL and C.conv_tail_ok(h1[..., cb:], lvl.cls[1], lvl.cls[2]):
            # class branch: 3x3 80 -> 80 + SiLU and the 1x1 80 -> 80 logits in one launch
            C.conv2d_tail(h1[..., cb:], lvl.cls[1], lvl.cls[2], out[..., 4 * REG_MAX:])
        else:
            C.conv2d(h1[..., cb:], lvl.cls[1], out=h2[..., cb:])
            C.conv2d(h2[..., cb:], lvl.cls[2], out=out[..., 4 * REG_MAX:])
        return out

    # ---- forward ------------------------------------------------------------------------------
    def letterbox(self, frame_hw):
        return V.letterbox_geometry(frame_hw[0], frame_hw[1], self.image_size)

    def preprocess(self, frames: torch.Tensor) -> torch.Tensor:
        """uint8 [B, H, W, 3] RGB -> letterboxed, /255, zero-bordered bf16 [B, Hp, Wp, 4]."""
        B, H, W, _ = frames.shape
        Ho, Wo, top, left, _ = self.letterbox((H, W))
        S = self.image_size
        Hp, Wp = C.stem_geometry(S, S, 3, 2, 1)
        return V.preprocess_frames(frames, (Ho, Wo), V.YOLO_MEAN, V.YOLO_STD,
                                   out=self._buf("input", (B, Hp, Wp, 4)), stem=(3, 2, 1),
                                   canvas=(S, S, top, left, 114.0))

    def stem_from_frames(self, frames: torch.Tensor) -> torch.Tensor:
        """uint8 [B, H, W, 3] -> the stem conv's output [B, S/2, S/2, c1] in ONE kernel
        (``stem_direct_kernel``: letterbox + /255 into LDS, direct 3x3/2 conv, bias, SiLU) —
        no bf16 canvas round trip through HBM, no 27 -> 64 K padding."""
        B, H, W, _ = frames.shape
        Ho, Wo, top, left, _ = self.letterbox((H, W))
        S = self.image_size
        h0, w0 = C.stem_out_hw(S, S, 3, 2, 1)
        if self._stem_w is None:
            self._stem_w = torch.zeros(self.l0.cout, 64, dtype=torch.bfloat16, device=self.l0.weight.device)
            self._derive_stem_w()
        out = self._buf("a0", (B, h0, w0, self.ch[0]))
        torch.ops.aiko.stem_direct_out(frames, self._stem_w, self.l0.bias, out,
                                       [Ho, Wo, S, S, top, left, 3, 2, 1, 2], 114.0,
                                       list(V.YOLO_MEAN), list(V.YOLO_STD), False)
        return out

    def head_outputs(self, x: torch.Tensor | None, a0: torch.Tensor | None = None, decode: bool = False):
        """Stem buffer (or the stem output ``a0``) -> per-level head outputs
        [B, H/s, W/s, 64 + nc] for s = 8, 16, 32.  ``decode``: the head branches decode in their
        epilogues instead (:meth:`_decode_fused_ok`) and this returns (boxes, scores, cls)."""
        B = (x if a0 is None else a0).shape[0]
        S = self.image_size
        c1, c2, c3, c4, c5 = self.ch
        h0, w0 = C.stem_out_hw(S, S, 3, 2, 1)
        s = [(h0, w0)]
        for _ in range(4):
            h, w = s[-1]
            s.append(((h - 1) // 2 + 1, (w - 1) // 2 + 1))
        (H1, W1), (H2, W2), (H3, W3), (H4, W4), (H5, W5) = s
        a2 = self._buf("a2", (B, H2, W2, c2))
        if a0 is None:
            a0 = C.conv2d(x, self.l0, out=self._buf("a0", (B, H1, W1, c1)), image_hw=(S, S))
        a1 = C.conv2d(a0, self.l1, out=self._buf("a1", (B, H2, W2, c2)))
        a2 = self._run_c2f("l2", self.l2, a1, a2)
        cat14 = self._buf("cat14", (B, H3, W3, c4 + c3))       # [up(l12) | l4]
        a3 = self._buf("a3", (B, H3, W3, c3))
        if (_HEAD_TAIL and not self._c2f_fused_ok(self.l4, a3, cat14[..., c4:])
                and C.conv_tail_ok(a2, self.l3, self.l4.cv1)):
            # l3 (3x3 / 2) with l4's cv1 (1x1 + SiLU) in its epilogue: a3 is never written
            cat4 = self._buf("l4.cat", (B, H3, W3, (2 + len(self.l4.m)) * self.l4.c))
            C.conv2d_tail(a2, self.l3, self.l4.cv1, cat4[..., :2 * self.l4.c])
            a4 = self._run_c2f("l4", self.l4, a3, cat14[..., c4:], cat=cat4)
        else:
            C.conv2d(a2, self.l3, out=a3)
            a4 = self._run_c2f("l4", self.l4, a3, cat14[..., c4:])
        cat11 = self._buf("cat11", (B, H4, W4, c5 + c4))       # [up(l9) | l6]
        a5 = self._buf("a5", (B, H4, W4, c4))
        if (_HEAD_TAIL and not self._c2f_fused_ok(self.l6, a5, cat11[..., c5:])
                and C.conv_tail_ok(a4, self.l5, self.l6.cv1)):
            # l5 (3x3 / 2) with l6's cv1 in its epilogue: a5 is never written
            cat6 = self._buf("l6.cat", (B, H4, W4, (2 + len(self.l6.m)) * self.l6.c))
            C.conv2d_tail(a4, self.l5, self.l6.cv1, cat6[..., :2 * self.l6.c])
            a6 = self._run_c2f("l6", self.l6, a5, cat11[..., c5:], cat=cat6)
        else:
            C.conv2d(a4, self.l5, out=a5)
            a6 = self._run_c2f("l6", self.l6, a5, cat11[..., c5:])
        a7 = C.conv2d(a6, self.l7, out=self._buf("a7", (B, H5, W5, c5)))
        a8 = self._run_c2f("l8", self.l8, a7, self._buf("a8", (B, H5, W5, c5)))
        cat20 = self._buf("cat20", (B, H5, W5, c4 + c5))       # [l19 | l9]
        a9 = self._run_sppf("l9", self.l9, a8, cat20[..., c4:])
        DT.upsample2x(a9, out=cat11[..., :c5])
        cat17 = self._buf("cat17", (B, H4, W4, c3 + c4))       # [l16 | l12]
        a12 = self._run_c2f("l12", self.l12, cat11, cat17[..., c3:])
        p3 = self._buf("p3", (B, H3, W3, c3))
        if _UP_INPLACE and self._c2f_fused_ok(self.l15, cat14, p3) and W3 == 2 * a12.shape[2]:
            # l15's fused C2f reads up(l12) straight from a12: the upsampled half of cat14 is
            # never materialised
            self._run_c2f("l15", self.l15, cat14, p3, xu=a12)
        else:
            DT.upsample2x(a12, out=cat14[..., :c4])
            self._run_c2f("l15", self.l15, cat14, p3)
        C.conv2d(p3, self.l16, out=cat17[..., :c3])
        p4 = self._run_c2f("l18", self.l18, cat17, self._buf("p4", (B, H4, W4, c4)))
        C.conv2d(p4, self.l19, out=cat20[..., :c4])
        p5 = self._run_c2f("l21", self.l21, cat20, self._buf("p5", (B, H5, W5, c5)))
        if decode:
            A = sum(p.shape[1] * p.shape[2] for p in (p3, p4, p5))
            boxes = self._buf("boxes", (B, A, 4), torch.float32)
            scores = self._buf("scores", (B, A), torch.float32)
            cls = self._buf("cls", (B, A), torch.int32)
            astart = 0
            for i, (lvl, p) in enumerate(zip(self.heads, (p3, p4, p5))):
                self._run_head_decode(i, lvl, p, boxes, scores, cls, STRIDES[i], astart)
                astart += p.shape[1] * p.shape[2]
            return boxes, scores, cls
        return [self._run_head(i, lvl, p) for i, (lvl, p) in enumerate(zip(self.heads, (p3, p4, p5)))]

    def _decode_fused_ok(self) -> bool:
        """Can every detect-head branch run as a tail launch with the decode in its epilogue
        (box: 4 x 16 DFL bins on the 64-channel branch; class: the 80-channel branch)?"""
        return (_HEAD_TAIL and _DECODE_FUSED and self.device.type == "cuda" and self.cb == 4 * REG_MAX == 64
                and self.cc == 80 and self.nc_pad == 80
                and all(lvl.box[1].cout == 64 and lvl.cls[1].cout == 80 and lvl.box[1].stride == 1
                        and lvl.cls[1].stride == 1 for lvl in self.heads))

    def _run_head_decode(self, i, lvl: DetectLevel, x, boxes, scores, cls, stride, astart):
        """Detect head level ``i`` straight to decoded (boxes, scores, cls) rows astart .. of
        the [B, A] outputs: the first conv, then each branch's 3x3 + 1x1 as one conv_glds tail
        launch whose epilogue decodes (box: DFL expectation -> xyxy; class: sigmoid(max) /
        argmax) — the [.., 64 + nc] head output is never written."""
        B, H, W, _ = x.shape
        cb = self.cb
        h1 = self._buf(f"h{i}.1", (B, H, W, cb + self.cc))
        C.conv2d(x, lvl.first, out=h1)
        zp = C.zero_page(x.device)
        for xs, (s1, s2), mode, nc in ((h1[..., :cb], (lvl.box[1], lvl.box[2]), 1, 4 * REG_MAX),
                                       (h1[..., cb:], (lvl.cls[1], lvl.cls[2]), 2, self.nc_pad)):
            if not C.conv_tail_ok(xs, s1, s2):
                raise ValueError("_run_head_decode: head branch not eligible for a tail launch")
            torch.ops.aiko.conv_glds_tail_decode_out(xs, s1.weight, s1.bias, s2.weight, s2.bias, boxes, scores, cls,
                                                     s1.R, s1.pad, s1.act, mode, nc, stride, astart, zp)

    def _nms(self, boxes, scores, cls, frame_hw):
        B = boxes.shape[0]
        _, _, top, left, gain = self.letterbox(frame_hw)
        return DT.topk_nms(boxes, scores, cls, self.conf, self.iou, self.max_candidates, self.max_det,
                           (gain, left, top, frame_hw[1], frame_hw[0]),
                           det=self._buf("det", (B, self.max_det, 6), torch.float32),
                           count=self._buf("count", (B,), torch.int32))

    def postprocess(self, feats, frame_hw):
        B = feats[0].shape[0]
        A = sum(f.shape[1] * f.shape[2] for f in feats)
        boxes, scores, cls = DT.yolo_decode(
            feats, STRIDES, self.nc_pad, boxes=self._buf("boxes", (B, A, 4), torch.float32),
            scores=self._buf("scores", (B, A), torch.float32), cls=self._buf("cls", (B, A), torch.int32))
        _, _, top, left, gain = self.letterbox(frame_hw)
        return DT.topk_nms(boxes, scores, cls, self.conf, self.iou, self.max_candidates, self.max_det,
                           (gain, left, top, frame_hw[1], frame_hw[0]),
                           det=self._buf("det", (B, self.max_det, 6), torch.float32),
                           count=self._buf("count", (B,), torch.int32))

    def detect(self, frames: torch.Tensor):
        H, W = frames.shape[1:3]
        if self.fused_stem and self._decode_fused_ok():
            return self._nms(*self.head_outputs(None, a0=self.stem_from_frames(frames), decode=True), (H, W))
        if self.fused_stem:
            return self.postprocess(self.head_outputs(None, a0=self.stem_from_frames(frames)), (H, W))
        return self.postprocess(self.head_outputs(self.preprocess(frames)), (H, W))

    __call__ = detect

    # ---- bookkeeping ----------------------------------------------------------------------------
    def named_layers(self):
        return self.conv_specs()

    def config(self) -> dict:
        return {"scale": self.scale, "num_classes": self.nc, "image_size": self.image_size}

    def _derive_stem_w(self):
        """bf16 [Cout, 64] direct-stem weight, k = (r * 3 + s) * 4 + c, from the packed stem —
        written into the existing tensor so captured hipGraphs see reloaded weights."""
        l0 = self.l0
        cc = l0.Cc
        wp = l0.weight[:, :3 * cc].reshape(l0.cout, 3, cc // 4, 4)[:, :, :3, :]   # [o][r][s][c4]
        self._stem_w.zero_()
        self._stem_w[:, :36] = wp.reshape(l0.cout, 36)

    def _weights_loaded(self):
        """Re-derive each head level's fused box|cls first conv (and the direct-stem weight)
        from the loaded layers, in place."""
        if self._stem_w is not None:
            self._derive_stem_w()
        for lvl in self.heads:
            a, b = lvl.box[0], lvl.cls[0]
            lvl.first.weight[:a.cout].copy_(a.weight)
            lvl.first.weight[a.cout:].copy_(b.weight)
            if lvl.first.bias is not None:
                lvl.first.bias[:a.cout].copy_(a.bias)
                lvl.first.bias[a.cout:].copy_(b.bias)

    def conv_specs(self):
        yield "l0", self.l0
        for name in ("l1", "l3", "l5", "l7", "l16", "l19"):
            yield name, getattr(self, name)
        for name in ("l2", "l4", "l6", "l8", "l12", "l15", "l18", "l21"):
            blk = getattr(self, name)
            yield f"{name}.cv1", blk.cv1
            yield f"{name}.cv2", blk.cv2
            for i, (a, b) in enumerate(blk.m):
                yield f"{name}.m{i}.cv1", a
                yield f"{name}.m{i}.cv2", b
        yield "l9.cv1", self.l9.cv1
        yield "l9.cv2", self.l9.cv2
        for i, lvl in enumerate(self.heads):
            for j, s in enumerate(lvl.box):
                yield f"head{i}.box{j}", s
            for j, s in enumerate(lvl.cls):
                yield f"head{i}.cls{j}", s

    def flops_per_image(self) -> int:
        total = 0
        S = self.image_size
        ref = self.reference_shapes()
        for name, spec in self.conv_specs():
            H, W = ref[name]
            total += spec.flops(1, H, W) if spec.kind != "stem" else spec.flops(1, S, S)
        return total

    def reference_shapes(self):
        """Input spatial size of every conv (for FLOP accounting)."""
        S = self.image_size
        sz = [S // 2, S // 4, S // 8, S // 16, S // 32]
        shapes = {"l0": (S, S), "l1": (sz[0],) * 2, "l3": (sz[1],) * 2, "l5": (sz[2],) * 2,
                  "l7": (sz[3],) * 2, "l16": (sz[2],) * 2, "l19": (sz[3],) * 2}
        where = {"l2": sz[1], "l4": sz[2], "l6": sz[3], "l8": sz[4], "l12": sz[3], "l15": sz[2],
                 "l18": sz[3], "l21": sz[4]}
        for name, s in where.items():
            blk = getattr(self, name)
            shapes[f"{name}.cv1"] = shapes[f"{name}.cv2"] = (s, s)
            for i in range(len(blk.m)):
                shapes[f"{name}.m{i}.cv1"] = shapes[f"{name}.m{i}.cv2"] = (s, s)
        shapes["l9.cv1"] = shapes["l9.cv2"] = (sz[4],) * 2
        for i, s in enumerate(sz[2:]):
            for j in range(3):
                shapes[f"head{i}.box{j}"] = shapes[f"head{i}.cls{j}"] = (s, s)
        return shapes

    # ---- fp32 torch reference (tests only) ----------------------------------------------------
    def reference_head_outputs(self, frames: torch.Tensor):
        import torch.nn.functional as F

        from ..ops import reference as R
        B, H, W, _ = frames.shape
        Ho, Wo, top, left, _ = self.letterbox((H, W))
        S = self.image_size
        x = frames.permute(0, 3, 1, 2).float()
        if (Ho, Wo) != (H, W):
            x = F.interpolate(x, size=(Ho, Wo), mode="bilinear", align_corners=False)
        canvas = torch.full((B, 3, S, S), 114.0, device=x.device)
        canvas[:, :, top:top + Ho, left:left + Wo] = x
        x = canvas / 255.0

        def c2f(blk, x):
            y = R.conv_ref(x, blk.cv1)
            ys = [y[:, :blk.c], y[:, blk.c:]]
            for a, b in blk.m:
                t = R.conv_ref(R.conv_ref(ys[-1], a), b, residual_nchw=ys[-1] if blk.shortcut else None,
                               residual_after_act=True)
                ys.append(t)
            return R.conv_ref(torch.cat(ys, 1), blk.cv2)

        def sppf(blk, x):
            y = [R.conv_ref(x, blk.cv1)]
            for _ in range(3):
                y.append(F.max_pool2d(y[-1], blk.k, 1, blk.k // 2))
            return R.conv_ref(torch.cat(y, 1), blk.cv2)

        up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")  # noqa: E731
        a0 = R.conv_ref(x, self.l0)
        a2 = c2f(self.l2, R.conv_ref(a0, self.l1))
        a4 = c2f(self.l4, R.conv_ref(a2, self.l3))
        a6 = c2f(self.l6, R.conv_ref(a4, self.l5))
        a9 = sppf(self.l9, c2f(self.l8, R.conv_ref(a6, self.l7)))
        a12 = c2f(self.l12, torch.cat([up(a9), a6], 1))
        p3 = c2f(self.l15, torch.cat([up(a12), a4], 1))
        p4 = c2f(self.l18, torch.cat([R.conv_ref(p3, self.l16), a12], 1))
        p5 = c2f(self.l21, torch.cat([R.conv_ref(p4, self.l19), a9], 1))
        outs = []
        for lvl, p in zip(self.heads, (p3, p4, p5)):
            bx = p
            for s in lvl.box:
                bx = R.conv_ref(bx, s)
            cl = p
            for s in lvl.cls:
                cl = R.conv_ref(cl, s)
            outs.append(torch.cat([bx, cl], 1))
        return outs
