"""Processing layer (mirror of src/processing): reader, per-cell API, cell processor."""
