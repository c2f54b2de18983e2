"""Host-side mirror of the reference's `pydata` package, limited to the FCD hot path's
callers: analyze.load_image, analyze.mask / center, analyze.folder."""
