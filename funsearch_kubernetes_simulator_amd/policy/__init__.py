"""policy subpackage."""
