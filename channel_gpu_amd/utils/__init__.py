"""Configuration, file I/O and timing utilities."""
