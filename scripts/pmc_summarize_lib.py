"""The step-kernel dispatch filter shared by the PMC summarisers."""
STEP_KERNELS = ("wave_kernel", "tile_kernel", "split_kernel", "block_kernel")


def is_step(name):
    """A step launch, not the observe-only instantiation (the OBS_ONLY
    template argument: 4th of split_kernel, 3rd of the others)."""
    if not any(k in name for k in STEP_KERNELS):
        return False
    args = name[name.index("<") + 1:name.index(">")].split(",")
    i = 3 if "split_kernel" in name else 2
    return len(args) > i and args[i].strip() == "false"
