/* rt_fastcall.c — a CPython binding of the one call on the timed path, rt_update_frames
 * (include/rt_abi.h), linked against librt_hip.so, so that the Python mirror of the plugin
 * (gpu_ray_tracing.ComputeShaderPipeline.bind_update_frames) issues it without ctypes'
 * per-argument conversion and numpy's __array_interface__ dictionaries: a ctypes call of
 * the 14-argument function with the arrays' addresses looked up costs ≈ 8.7 µs of host
 * time on the build container's CPU (0.3 µs through this binding), all of it before the
 * call's first launch reaches the GPU; on the GPU boxes' EPYC the difference measured
 * ≈ 2 µs per call (profiles/r05/r05b_region_k3.jsonl, DESIGN.md §5 "Fixed cost of a call").
 *
 *   update_frames(ctx, a, b, w, h, rank, nranks, camera, spheres, count, seeds, stream)
 *       -> newest image (0 / 1), or -status when the library returns an error
 *
 * ctx, a, b and stream are the addresses the ctypes binding passes (the context handle
 * from rt_create, device image pointers, the HIP stream); camera, spheres and seeds are
 * objects exporting C-contiguous float32 buffers (numpy arrays).  Anything else raises
 * TypeError and the caller converts.  No HIP call here: the library does all of that. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

#include "rt_abi.h"

static int f32_buffer(PyObject* o, Py_buffer* b, const char* what) {
    if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) return -1;
    if (b->itemsize != 4 || !b->format || strcmp(b->format, "f") != 0) {
        PyBuffer_Release(b);
        PyErr_Format(PyExc_TypeError, "%s must be C-contiguous float32", what);
        return -1;
    }
    return 0;
}

static PyObject* update_frames(PyObject* self, PyObject* const* args, Py_ssize_t n) {
    (void)self;
    if (n != 12) {
        PyErr_SetString(PyExc_TypeError, "update_frames takes 12 arguments");
        return NULL;
    }
    void* addr[3];
    for (int i = 0; i < 3; ++i) {                /* ctx, a, b */
        addr[i] = PyLong_AsVoidPtr(args[i]);
        if (!addr[i] && PyErr_Occurred()) return NULL;
    }
    uint32_t u[5];
    const int u_at[5] = {3, 4, 5, 6, 9};         /* w, h, rank, nranks, count */
    for (int i = 0; i < 5; ++i) {
        const unsigned long v = PyLong_AsUnsignedLong(args[u_at[i]]);
        if (v == (unsigned long)-1 && PyErr_Occurred()) return NULL;
        if (v > 0xFFFFFFFFul) {
            PyErr_SetString(PyExc_OverflowError, "argument does not fit uint32");
            return NULL;
        }
        u[i] = (uint32_t)v;
    }
    void* stream = args[11] == Py_None ? NULL : PyLong_AsVoidPtr(args[11]);
    if (!stream && PyErr_Occurred()) return NULL;
    Py_buffer cam, sph, seeds;
    if (f32_buffer(args[7], &cam, "camera") != 0) return NULL;
    if (cam.len != (Py_ssize_t)sizeof(rt_scene_camera)) {
        PyBuffer_Release(&cam);
        PyErr_SetString(PyExc_TypeError, "camera must be the 176-byte SceneCamera blob");
        return NULL;
    }
    if (f32_buffer(args[8], &sph, "spheres") != 0) {
        PyBuffer_Release(&cam);
        return NULL;
    }
    if ((size_t)sph.len < (size_t)u[4] * sizeof(rt_sphere)) {
        PyBuffer_Release(&cam);
        PyBuffer_Release(&sph);
        PyErr_SetString(PyExc_ValueError, "spheres holds fewer than count records");
        return NULL;
    }
    if (f32_buffer(args[10], &seeds, "seeds") != 0) {
        PyBuffer_Release(&cam);
        PyBuffer_Release(&sph);
        return NULL;
    }
    int newest = -1;
    rt_status st;
    /* (the GIL released while the library issues the launches, as ctypes does: the held
     * buffers keep the arrays alive) */
    Py_BEGIN_ALLOW_THREADS
    st = rt_update_frames((rt_ctx*)addr[0], (float*)addr[1], (float*)addr[2], u[0], u[1], u[2],
                          u[3], (const rt_scene_camera*)cam.buf, (const rt_sphere*)sph.buf, u[4],
                          (uint32_t)(seeds.len / 4), (const float*)seeds.buf, stream, &newest);
    Py_END_ALLOW_THREADS
    PyBuffer_Release(&cam);
    PyBuffer_Release(&sph);
    PyBuffer_Release(&seeds);
    return PyLong_FromLong(st ? -(long)st : (long)newest);
}

static PyMethodDef methods[] = {
    {"update_frames", (PyCFunction)(void (*)(void))update_frames, METH_FASTCALL,
     "rt_update_frames: newest image, or -status"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_rt_fastcall",
                                    "rt_update_frames without ctypes (rt_fastcall.c)", -1,
                                    methods};

PyMODINIT_FUNC PyInit__rt_fastcall(void) { return PyModule_Create(&module); }
