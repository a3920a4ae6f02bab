"""Config-file entry points (the north star's "YAML-config / src/engine trainer entry")."""
