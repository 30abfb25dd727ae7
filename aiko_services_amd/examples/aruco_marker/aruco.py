"""ArUco-style square marker detection and overlay (reference ``examples/aruco_marker/aruco.py:80-185``).

``ArucoMarkerDetector`` uses ``cv2.aruco`` (dictionary ``DICT_4X4_50``, parameter ``aruco_tags``)
when OpenCV is installed.  OpenCV is not in this image, so the element falls back to a small
numpy / scipy detector for axis-aligned markers: dark connected components -> square bounding
box -> border check -> the bit grid read in all four rotations.  Two codings:

* ``aruco_tags: DICT_ARUCO_ORIGINAL`` — the original ArUco markers (7x7 cells: a black border
  around 5x5 bits).  Every row is one of the four codewords 10000, 10111, 01001, 01110 (white =
  1, first column = most significant bit); columns 1 and 3 carry two id bits per row, row 0
  first, so ids 0..1023 are decoded exactly and a grid whose rows are not all codewords in any
  rotation is rejected.  The orientation is the first rotation that decodes.  Matching cv2's
  ``DICT_ARUCO_ORIGINAL`` table itself is unpinned here (no OpenCV to compare against).
* any other ``aruco_tags`` (default ``DICT_4X4_50``): 6x6-cell markers with a 16-bit payload;
  the id is the smallest payload over the rotations (rotation invariant), not the OpenCV
  dictionary index — the predefined 4x4..7x7 tables are OpenCV data, not derivable: documented
  parity gap.

Output per image: ``{"corners": [array(1, 4, 2)], "ids": array(N, 1)}`` as in OpenCV, corners
ordered top-left, top-right, bottom-right, bottom-left of the marker's own frame.

``ArucoMarkerOverlay`` draws each marker's outline, centre and id (PIL instead of cv2).
``make_marker(code, cell)`` / ``make_marker_original(marker_id, cell)`` render markers (tests,
demos).
"""
from __future__ import annotations

import numpy as np
from PIL import Image, ImageDraw

from ...elements.media.image_io import to_numpy_rgb
from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent

__all__ = ["ArucoMarkerDetector", "ArucoMarkerOverlay", "detect_markers_numpy", "make_marker",
           "make_marker_original", "decode_original"]

try:  # optional
    import cv2  # noqa: F401
    _CV2 = hasattr(cv2, "aruco")
except ImportError:
    cv2 = None
    _CV2 = False

COLOR_BOX = (255, 255, 0)
COLOR_CIRCLE = (255, 0, 0)
COLOR_TEXT = (255, 0, 255)
GRID = 6                      # cells per side including the border (16-bit payload markers)
GRID_ORIGINAL = 7             # DICT_ARUCO_ORIGINAL: border + 5x5 bits
_ORIGINAL_WORDS = (0x10, 0x17, 0x09, 0x0E)   # row codeword for 2 id bits 00, 01, 10, 11


def make_marker(code: int, cell: int = 8, quiet: int = 1) -> np.ndarray:
    """uint8 grayscale image of the 4x4 payload ``code`` (bit i = row i // 4, col i % 4,
    1 = white) with a black border and ``quiet`` white cells around it."""
    n = GRID + 2 * quiet
    grid = np.ones((n, n), np.uint8) * 255
    grid[quiet:quiet + GRID, quiet:quiet + GRID] = 0
    for i in range(16):
        if (code >> i) & 1:
            grid[quiet + 1 + i // 4, quiet + 1 + i % 4] = 255
    return np.kron(grid, np.ones((cell, cell), np.uint8))


def original_bits(marker_id: int) -> np.ndarray:
    """5x5 bits (1 = white) of original-ArUco marker ``marker_id`` (0..1023)."""
    if not 0 <= marker_id < 1024:
        raise ValueError(f"DICT_ARUCO_ORIGINAL ids are 0..1023 (got {marker_id})")
    bits = np.zeros((5, 5), np.uint8)
    for y in range(5):
        word = _ORIGINAL_WORDS[(marker_id >> 2 * (4 - y)) & 3]
        for x in range(5):
            bits[y, x] = (word >> (4 - x)) & 1
    return bits


def make_marker_original(marker_id: int, cell: int = 8, quiet: int = 1) -> np.ndarray:
    """uint8 grayscale image of original-ArUco marker ``marker_id`` with ``quiet`` white cells."""
    n = GRID_ORIGINAL + 2 * quiet
    grid = np.ones((n, n), np.uint8) * 255
    grid[quiet:quiet + GRID_ORIGINAL, quiet:quiet + GRID_ORIGINAL] = 0
    grid[quiet + 1:quiet + 6, quiet + 1:quiet + 6] = original_bits(marker_id) * 255
    return np.kron(grid, np.ones((cell, cell), np.uint8))


def decode_original(bits: np.ndarray):
    """Id of a 5x5 bit grid (1 = white) in its own orientation, or None if a row is not a
    codeword."""
    marker_id = 0
    for y in range(5):
        word = int(sum(int(bits[y, x]) << (4 - x) for x in range(5)))
        if word not in _ORIGINAL_WORDS:
            return None
        marker_id = (marker_id << 2) | (int(bits[y, 1]) << 1) | int(bits[y, 3])
    return marker_id


def _code(bits: np.ndarray) -> int:
    return int(sum(int(b) << i for i, b in enumerate(bits.reshape(-1))))


def detect_markers_numpy(image, min_side: int = 12, dictionary: str = "DICT_4X4_50"):
    """Axis-aligned marker detector: returns (corners list of [1, 4, 2] float32, ids [N, 1]).
    ``dictionary`` ``DICT_ARUCO_ORIGINAL`` decodes original-ArUco ids; anything else reads the
    16-bit payload markers of ``make_marker``."""
    from scipy import ndimage
    original = str(dictionary) == "DICT_ARUCO_ORIGINAL"
    grid_n = GRID_ORIGINAL if original else GRID
    g = to_numpy_rgb(image)
    g = g.mean(axis=2) if g.ndim == 3 else g.astype(np.float64)
    thresh = 0.5 * (float(g.min()) + float(g.max()))
    dark = g < thresh
    labels, n = ndimage.label(dark)
    corners, ids = [], []
    for sl in ndimage.find_objects(labels):
        if sl is None:
            continue
        y0, y1, x0, x1 = sl[0].start, sl[0].stop, sl[1].start, sl[1].stop
        h, w = y1 - y0, x1 - x0
        if min(h, w) < min_side or abs(h - w) > 0.15 * max(h, w):
            continue
        # sample the centre of every cell of the grid
        cy = y0 + (np.arange(grid_n) + 0.5) * h / grid_n
        cx = x0 + (np.arange(grid_n) + 0.5) * w / grid_n
        cells = dark[cy.astype(int)[:, None], cx.astype(int)[None, :]]
        border = np.concatenate([cells[0], cells[-1], cells[:, 0], cells[:, -1]])
        if not border.all():
            continue
        bits = ~cells[1:-1, 1:-1]                       # white = 1
        rots = [np.rot90(bits, -k) for k in range(4)]   # marker rotated k quarter turns clockwise
        if original:
            decoded = [decode_original(r) for r in rots]
            found = [k for k in range(4) if decoded[k] is not None]
            if not found:
                continue
            k = found[0]
            marker_id = decoded[k]
        else:
            codes = [_code(r) for r in rots]
            k = int(np.argmin(codes))
            marker_id = codes[k]
        quad = np.array([[x0, y0], [x1, y0], [x1, y1], [x0, y1]], np.float32)
        # the marker's own top-left corner after undoing k clockwise quarter turns
        quad = np.roll(quad, -((4 - k) % 4), axis=0)
        corners.append(quad.reshape(1, 4, 2))
        ids.append([marker_id])
    return corners, np.array(ids, np.int32).reshape(-1, 1)


class ArucoMarkerDetector(PipelineElement):
    def __init__(self, context):
        context.set_protocol("aruco_marker_detector:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self._detector = None
        tags, _ = self.get_parameter("aruco_tags", "DICT_4X4_50")
        self._tags = str(tags)
        if _CV2:
            dictionary = cv2.aruco.getPredefinedDictionary(getattr(cv2.aruco, self._tags))
            self._detector = cv2.aruco.ArucoDetector(dictionary, cv2.aruco.DetectorParameters())

    def process_frame(self, stream, images):
        overlays = []
        for image in images:
            if self._detector is not None:
                corners, ids, _ = self._detector.detectMarkers(to_numpy_rgb(image))
                ids = np.zeros((0, 1), np.int32) if ids is None else ids
            else:
                corners, ids = detect_markers_numpy(image, dictionary=self._tags)
            overlays.append({"corners": list(corners), "ids": ids})
        return StreamEvent.OKAY, {"overlays": overlays}


class ArucoMarkerOverlay(PipelineElement):
    def __init__(self, context):
        context.set_protocol("aruco_marker_overlay:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, images, overlays):
        out = []
        for image, overlay in zip(images, overlays):
            arr = to_numpy_rgb(image)
            corners, ids = overlay.get("corners", []), np.asarray(overlay.get("ids", [])).reshape(-1)
            if len(corners):
                pil = Image.fromarray(arr.astype(np.uint8)).convert("RGB")
                draw = ImageDraw.Draw(pil)
                for quad, marker_id in zip(corners, ids):
                    pts = [tuple(int(v) for v in p) for p in np.asarray(quad).reshape(4, 2)]
                    draw.line(pts + [pts[0]], fill=COLOR_BOX, width=2)
                    cx = (pts[0][0] + pts[2][0]) // 2
                    cy = (pts[0][1] + pts[2][1]) // 2
                    draw.ellipse([cx - 4, cy - 4, cx + 4, cy + 4], fill=COLOR_CIRCLE)
                    draw.text((pts[0][0], max(0, pts[0][1] - 15)), str(int(marker_id)), fill=COLOR_TEXT)
                arr = np.asarray(pil)
            out.append(arr)
        return StreamEvent.OKAY, {"images": out, "overlays": overlays}
