"""Reference plugin path mirror: ``importlib.import_module("model.NRMS")``
(src/train.py:18, src/evaluate.py:15) resolves here when this directory's
parent is on sys.path."""
