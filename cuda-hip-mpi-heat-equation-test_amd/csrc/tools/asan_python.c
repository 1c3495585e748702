/* A Python interpreter with AddressSanitizer's runtime linked in first, so
 * that the whole process — CPython (PYTHONMALLOC=malloc), numpy, torch and an
 * ASan-instrumented libheat2d.so loaded through HEAT2D_LIB — allocates through
 * ASan's malloc: the ctypes boundary, the transports' callbacks and the
 * runtime's host code run under heap checks without any preloading
 * (`make asan-python`, tests/test_sanitizers.py). */
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
