"""gym 0.21 registration stand-in: records ids only (fixture generation only)."""
registry = {}


def register(id, entry_point=None, **kwargs):
    registry[id] = entry_point
