"""Minimal stand-in for gym 0.15.7 (absent from this image) used only to import the
reference env modules while generating golden vectors. Env is a plain base class;
register/make are no-ops. Written for this repo; not gym source."""
from . import spaces  # noqa: F401


class Env(object):
    def __init__(self, *args, **kwargs):
        pass


def register(*args, **kwargs):
    return None


def make(*args, **kwargs):
    raise NotImplementedError("gym stub: make() is not available")
