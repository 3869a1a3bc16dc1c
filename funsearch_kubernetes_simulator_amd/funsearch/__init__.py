"""funsearch subpackage."""
