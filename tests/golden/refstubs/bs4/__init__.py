class BeautifulSoup:
    """Import-only stand-in (VeRi XML parsing, never called)."""

    def __init__(self, *args, **kwargs):
        raise RuntimeError("bs4 is unavailable offline")
