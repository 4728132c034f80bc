from . import env, logging  # noqa: F401
