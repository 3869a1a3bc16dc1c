"""bench subpackage."""
