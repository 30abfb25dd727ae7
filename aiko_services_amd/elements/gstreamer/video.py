"""GStreamer readers / writers (reference ``elements/gstreamer/video_*.py``)."""
from __future__ import annotations

import queue
import threading

import numpy as np

from . import utilities as U

__all__ = ["VideoReader", "VideoFileReader", "VideoCameraReader", "VideoStreamReader",
           "VideoFileWriter", "VideoStreamWriter", "file_reader_launch", "camera_reader_launch",
           "stream_reader_launch", "file_writer_launch", "stream_writer_launch"]


# ---- launch descriptions (pure, testable without GStreamer) ---------------------------------

def file_reader_launch(filename: str) -> str:
    return (f"filesrc location={filename} ! qtdemux ! {U.get_h264_decoder()} ! videoconvert ! "
            f"video/x-raw, format={U.get_format()} ! appsink name=sink")


def camera_reader_launch(devicepath: str) -> str:
    return (f"v4l2src device={devicepath} ! videoflip video-direction=horiz ! videoconvert ! "
            f"videorate ! video/x-raw, format={U.get_format()} ! appsink name=sink")


def stream_reader_launch(hostname: str, port: int, rtp: bool = True) -> str:
    if rtp:
        return (f'udpsrc address={hostname} port={port} caps="application/x-rtp, media=video, '
                f'encoding-name=H264, payload=96" ! rtph264depay ! h264parse ! {U.get_h264_decoder()} ! '
                f"videoconvert ! video/x-raw, format={U.get_format()} ! appsink name=sink")
    return (f"tcpclientsrc host={hostname} port={port} ! decodebin ! videoconvert ! "
            f"video/x-raw, format={U.get_format()} ! appsink name=sink")


def file_writer_launch(filename: str, width: int, height: int, framerate: int) -> str:
    return (f"appsrc name=source ! videoconvert ! videoscale ! videorate ! "
            f"video/x-raw,width={width},height={height},framerate={framerate}/1 ! "
            f"{U.get_h264_encoder()} ! splitmuxsink location={filename}")


def stream_writer_launch(hostname: str, port: int, rtmp_url: str | None = None) -> str:
    if rtmp_url:
        return ("appsrc name=source ! videoconvert ! x264enc bitrate=1000 me=4 subme=10 ref=2 "
                "tune=zerolatency ! video/x-h264 ! h264parse ! video/x-h264 ! queue ! "
                f'flvmux name=muxer streamable=true ! rtmpsink location="{rtmp_url}" sync=false')
    return (f"appsrc name=source ! videoconvert ! {U.get_h264_encoder()} {U.get_h264_encoder_options()} ! "
            f"rtph264pay config-interval=5 pt=96 ! udpsink host={hostname} port={port}")


# ---- readers --------------------------------------------------------------------------------

class VideoReader:
    """Runs a launch description ending in ``appsink name=sink``; samples -> frame queue."""

    def __init__(self, launch: str, width: int | None = None, height: int | None = None):
        self.Gst = U.gst_initialise()
        self.launch = launch
        self.queue: queue.Queue = queue.Queue()
        self.frame_id = 0
        self.finished = False
        self.pipeline = self.Gst.parse_launch(launch)
        sink = self.pipeline.get_by_name("sink")
        sink.set_property("emit-signals", True)
        sink.connect("new-sample", self.sample_image, None)
        bus = self.pipeline.get_bus()
        self.pipeline.set_state(self.Gst.State.PLAYING)
        threading.Thread(target=self._run, args=(bus,), daemon=True).start()

    def _run(self, bus):
        Gst = self.Gst
        while True:
            msg = bus.timed_pop_filtered(Gst.CLOCK_TIME_NONE, Gst.MessageType.ERROR | Gst.MessageType.EOS)
            if msg is not None:
                self.finished = True
                self.queue.put({"type": "EOS" if msg.type == Gst.MessageType.EOS else "error"})
                self.pipeline.set_state(Gst.State.NULL)
                return

    def gst_to_numpy(self, sample) -> np.ndarray:
        buf = sample.get_buffer()
        caps = sample.get_caps().get_structure(0)
        h, w = caps.get_value("height"), caps.get_value("width")
        data = buf.extract_dup(0, buf.get_size())
        return np.frombuffer(data, np.uint8).reshape(h, w, -1)[..., :3].copy()

    def sample_image(self, sink, _data):
        sample = sink.emit("pull-sample")
        self.queue.put({"type": "image", "id": self.frame_id, "image": self.gst_to_numpy(sample)})
        self.frame_id += 1
        return self.Gst.FlowReturn.OK

    def read_frame(self, timeout=None):
        try:
            return self.queue.get(timeout=timeout)
        except queue.Empty:
            return None

    def queue_size(self):
        return self.queue.qsize()


class VideoFileReader(VideoReader):
    def __init__(self, input_filename, width=None, height=None):
        super().__init__(file_reader_launch(input_filename), width, height)


class VideoCameraReader(VideoReader):
    def __init__(self, input_devicepath, width=None, height=None):
        super().__init__(camera_reader_launch(input_devicepath), width, height)


class VideoStreamReader(VideoReader):
    def __init__(self, input_hostname, input_port, width=None, height=None, rtp=True):
        super().__init__(stream_reader_launch(input_hostname, input_port, rtp), width, height)


# ---- writers --------------------------------------------------------------------------------

class _Writer:
    def __init__(self, launch: str, width: int, height: int, framerate: int):
        self.Gst = U.gst_initialise()
        self.launch = launch
        self.width, self.height, self.framerate = width, height, framerate
        self.queue: queue.Queue = queue.Queue()
        self.pipeline = self.Gst.parse_launch(launch)
        self.source = self.pipeline.get_by_name("source")
        caps = self.Gst.Caps.from_string(
            f"video/x-raw,format={U.get_format()},width={width},height={height},framerate={framerate}/1")
        self.source.set_property("caps", caps)
        self.source.set_property("format", self.Gst.Format.TIME)
        self.pipeline.set_state(self.Gst.State.PLAYING)
        self.frame_count = 0
        threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        Gst = self.Gst
        duration = Gst.SECOND // max(1, self.framerate)
        while True:
            frame = self.queue.get()
            if frame is None:
                self.source.emit("end-of-stream")
                return
            image = np.ascontiguousarray(frame["image"], dtype=np.uint8)
            buf = Gst.Buffer.new_wrapped(image.tobytes())
            buf.pts = self.frame_count * duration
            buf.duration = duration
            self.frame_count += 1
            self.source.emit("push-buffer", buf)

    def write_frame(self, frame):
        self.queue.put(frame)

    def queue_size(self):
        return self.queue.qsize()

    def close(self):
        self.queue.put(None)


class VideoFileWriter(_Writer):
    def __init__(self, filename, width, height, framerate):
        super().__init__(file_writer_launch(filename, width, height, framerate), width, height, framerate)


class VideoStreamWriter(_Writer):
    def __init__(self, hostname, port, width, height, framerate, rtmp_url=None):
        super().__init__(stream_writer_launch(hostname, port, rtmp_url), width, height, framerate)
