"""pyfcd — MI355X-native drop-in for the reference's pyfcd package.

Same module layout as /root/reference/pyfcd (fcd.py, fourier.py, carriers.py);
the compute runs in lib/libfcd_mi355x.so (HIP kernels for gfx950).
"""
