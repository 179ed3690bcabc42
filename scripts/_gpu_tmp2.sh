timeout -k 10 300 python scripts/rt_ab16.py "" computer-graphics_amd/_build_noshade/libcgamd.so computer-graphics_amd/_build_noshadow/libcgamd.so
CGAMD_LIB=$PWD/computer-graphics_amd/_build_stamps/libcgamd.so CG_RT_LAT_DIAG=1 timeout -k 10 100 python bench.py --steps 32 --warmup 16 --no-cpu-baseline 2>&1 | grep "cycles per wave" | tail -1
