"""Utilities: design-rule post-processing, results I/O, environment reporting."""
