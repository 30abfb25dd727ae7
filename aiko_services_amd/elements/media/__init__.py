"""Media element library (reference ``elements/media/__init__.py``)."""
from .common_io import DataSource, DataTarget, contains_all, file_glob_difference  # noqa: F401
from .audio_io import (AudioFraming, AudioOutput, AudioReadFile, AudioResampler,  # noqa: F401
                       AudioSynthetic, AudioWriteFile, PE_FFT)
from .image_io import ImageOutput, ImageOverlay, ImageReadFile, ImageResize, ImageWriteFile  # noqa: F401
from .text_io import TextOutput, TextReadFile, TextSample, TextTransform, TextWriteFile  # noqa: F401
from .video_io import (VideoOutput, VideoReadFile, VideoReadWebcam, VideoSample, VideoShow,  # noqa: F401
                       VideoWriteFile)
