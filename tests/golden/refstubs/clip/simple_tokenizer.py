class SimpleTokenizer:
    """Import-only stand-in (the BPE vocabulary file is absent offline)."""

    def __init__(self, *args, **kwargs):
        pass
