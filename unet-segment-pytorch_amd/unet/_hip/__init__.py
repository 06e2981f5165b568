"""HIP (gfx950) execution layer: ctypes binding (lib), runtime helpers, stage plans, autograd glue."""
