from .sgd import SGD  # noqa: F401
