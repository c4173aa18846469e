// heat3d-mi355x — cpu_rows.cpp built with -mfma -mavx2 (hardware FMA,
// vectorised); selected at run time by cpu_row_kernels().
#define H3D_ROWS_NS rows_fma
#include "cpu_rows.cpp"
