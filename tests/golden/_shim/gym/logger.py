"""gym 0.21 logger stand-in (fixture generation only)."""


def warn(msg, *args):
    pass


def info(msg, *args):
    pass
