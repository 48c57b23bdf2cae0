"""Library operations built on the AOT gfx950 kernels."""
