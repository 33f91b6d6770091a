"""Reference import name ``garfieldpp`` -> garfield_amd.runtime (see compat/README.md)."""
