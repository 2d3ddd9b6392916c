"""Stub: the reference imports ffmpeg-python only for load_audio(path); golden vectors feed arrays."""
