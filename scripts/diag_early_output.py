#!/usr/bin/env python3
"""Does the adaptive early output fire on the bench's path?  Renders C3 adaptive
through rtx_render_multi into a torch-pinned framebuffer (the bench's SharedFrame at N = 1), with
the default phases and with forced small ones, and prints rtx_internal_early_output_stats before
and after, plus what the HIP runtime reports for the buffer (hipPointerGetAttributes type,
hipHostGetDevicePointer)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3360-ray-tracer_amd"))


def main():
    import torch

    torch.cuda.init()
    import rtx

    hip = C.CDLL("libamdhip64.so")
    host = rtx.HostScene.recipe("bunny", 1234)
    dev = rtx.DeviceScene(host, device=0)
    for width in (1000, 120):
        cam = rtx.camera(rtx.camera_config("c3_bunny", width=width))
        npix = cam.image_width * cam.image_height
        out = torch.empty((npix, 3), dtype=torch.float64).pin_memory()
        attr = (C.c_int * 16)()
        rc = hip.hipPointerGetAttributes(C.byref(attr), C.c_void_p(out.data_ptr()))
        dp = C.c_void_p()
        rc2 = hip.hipHostGetDevicePointer(C.byref(dp), C.c_void_p(out.data_ptr()), 0)
        print(f"width {width}: hipPointerGetAttributes rc {rc} type {attr[0]}; hipHostGetDevicePointer rc {rc2} "
              f"{'mapped' if dp.value else 'none'}", flush=True)
        for knobs in ({}, dict(phase_slots=64, phase_kcap=8)):
            rtx.adapt_tune(**knobs)
            n0, p0 = rtx.early_output_stats()
            rtx.render_multi([dev], cam, 200, 20, seed=33, adaptive=True, out=out.numpy())
            n1, p1 = rtx.early_output_stats()
            print(f"  knobs {knobs}: early outputs {n1 - n0}, pixels patched {p1 - p0}", flush=True)
        rtx.adapt_tune()


if __name__ == "__main__":
    main()
