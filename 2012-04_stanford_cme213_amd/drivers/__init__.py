"""Command-line drivers (``python -m cme213x.drivers.<name>``)."""
