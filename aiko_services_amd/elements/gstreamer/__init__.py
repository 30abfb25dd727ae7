"""GStreamer video readers / writers (reference ``elements/gstreamer/``, whose own package
import was broken: ``from aiko_services.gstreamer import *``).

The GStreamer launch descriptions are built by pure functions (``*_launch``) and run through
``Gst.parse_launch`` with an ``appsink`` (readers: frames pulled into a queue by a thread) or an
``appsrc`` (writers: frames pushed from a queue).  PyGObject is installed in this image but the
Gst typelib is not, so constructing a reader/writer raises :class:`GStreamerError` here; on a
host with GStreamer the same classes work.  Frames are ``{"type": "image", "id": n, "image":
HxWx3 uint8 RGB}`` dictionaries as in the reference.
"""
from .utilities import (GStreamerError, enable_opencv, get_format, get_h264_decoder,  # noqa: F401
                        get_h264_encoder, get_h264_encoder_options, gst_initialise, process_video)
from .video import (VideoCameraReader, VideoFileReader, VideoFileWriter, VideoReader,  # noqa: F401
                    VideoStreamReader, VideoStreamWriter, camera_reader_launch, file_reader_launch,
                    file_writer_launch, stream_reader_launch, stream_writer_launch)
