"""Minimal no-op stand-in for ``loguru`` (absent from this image), used only by
tools/make_goldens.py so the reference modules import. Not product code."""


class _Logger:
    def __getattr__(self, name):
        return lambda *args, **kwargs: None


logger = _Logger()
