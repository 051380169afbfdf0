"""Reference-compatible command-line front ends (``python -m streamml.cli``)."""
