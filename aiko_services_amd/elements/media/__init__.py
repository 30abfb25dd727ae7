"""Media element library (reference ``elements/media/__init__.py``)."""
from .common_io import DataSource, DataTarget, contains_all, file_glob_difference  # noqa: F401
from .audio_io import (AudioFraming, AudioOutput, AudioReadFile, AudioResampler,  # noqa: F401
                       AudioSynthetic, AudioWriteFile, PE_AudioFilter, PE_AudioResampler, PE_FFT,
                       PE_GraphXY, PE_MicrophonePA, PE_MicrophoneSD, PE_RemoteReceive0,
                       PE_RemoteReceive1, PE_RemoteReceive2, PE_RemoteSend0, PE_RemoteSend1,
                       PE_RemoteSend2, PE_Speaker)
from .image_io import ImageOutput, ImageOverlay, ImageReadFile, ImageResize, ImageWriteFile  # noqa: F401
from .text_io import TextOutput, TextReadFile, TextSample, TextTransform, TextWriteFile  # noqa: F401
from .video_io import (VideoOutput, VideoReadFile, VideoReadWebcam, VideoSample, VideoShow,  # noqa: F401
                       VideoWriteFile)
