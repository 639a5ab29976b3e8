class RandomErasing:
    """Import-only stand-in (training transform, never called)."""

    def __init__(self, *args, **kwargs):
        pass
