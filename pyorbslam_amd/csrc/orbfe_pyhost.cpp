// pyorbslam_amd._pyhost: the per-frame Python objects the reference data model needs, built in C instead of
// Python loops (the C3 tracking loop's host time).  No computation: the values are the ones the
// GPU path produced; only the object construction moves out of the interpreter.
//   keypoint_tuples(kps)      the caster's cv::KeyPoint tuples (opencv_type_casters.h:106-108) from the
//                             extractor's (n,) orbfe_keypoint records: (x, y, size, angle, response) as Python
//                             floats (the exact f32 values) and octave as an int
//   grid_lists(flat, off, cols, rows)
//                             Frame.mGrid (Frame.py:143-159): cols lists of rows lists, cell (ix, iy) holding
//                             the ints flat[off[ix * rows + iy] : off[ix * rows + iy + 1]] (a new list per cell)
//   grid_assign(pts, min_x, min_y, w_inv, h_inv, cols, rows)
//                             the grid cells of every keypoint (pos_in_grid) and grid_lists of them, plus the CSR
//                             arrays
//   stereo_lists(u, depth, status, x, mbf)
//                             Frame.mvuRight / mvDepth (Frame.py:161-279) with the reference's element types:
//                             status 0 -> int -1; 1 -> np.float32 (u, depth); 2 -> Python floats x - 0.01 and
//                             mbf / 0.01 (the zero-disparity substitution in double)
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Kp {  // orbfe_keypoint (include/orbfe.h)
    float x, y, size, angle, response;
    int32_t octave;
};
static_assert(sizeof(Kp) == 24, "orbfe_keypoint layout");

// a C-contiguous 1-D array of the given item size, or an exception
bool contiguous(PyArrayObject* a, int itemsize, const char* what) {
    if (PyArray_NDIM(a) != 1 || !PyArray_IS_C_CONTIGUOUS(a) || PyArray_ITEMSIZE(a) != itemsize) {
        PyErr_Format(PyExc_ValueError, "%s: expected a contiguous 1-D array of %d-byte items", what, itemsize);
        return false;
    }
    return true;
}

PyObject* keypoint_tuples(PyObject*, PyObject* args) {
    PyArrayObject* a;
    if (!PyArg_ParseTuple(args, "O!", &PyArray_Type, &a) || !contiguous(a, (int)sizeof(Kp), "kps")) return nullptr;
    const npy_intp n = PyArray_DIM(a, 0);
    const Kp* k = (const Kp*)PyArray_DATA(a);
    PyObject* out = PyList_New(n);
    if (!out) return nullptr;
    for (npy_intp i = 0; i < n; ++i) {
        PyObject* t = PyTuple_New(6);
        if (!t) {
            Py_DECREF(out);
            return nullptr;
        }
        PyList_SET_ITEM(out, i, t);
        const float f[5] = {k[i].x, k[i].y, k[i].size, k[i].angle, k[i].response};
        for (int j = 0; j < 5; ++j) {
            PyObject* v = PyFloat_FromDouble((double)f[j]);
            if (!v) {
                Py_DECREF(out);
                return nullptr;
            }
            PyTuple_SET_ITEM(t, j, v);
        }
        PyObject* o = PyLong_FromLong(k[i].octave);
        if (!o) {
            Py_DECREF(out);
            return nullptr;
        }
        PyTuple_SET_ITEM(t, 5, o);
    }
    return out;
}

PyObject* grid_lists(PyObject*, PyObject* args) {
    PyArrayObject *flat, *off;
    int cols, rows;
    if (!PyArg_ParseTuple(args, "O!O!ii", &PyArray_Type, &flat, &PyArray_Type, &off, &cols, &rows) ||
        !contiguous(flat, 4, "flat") || !contiguous(off, 4, "off"))
        return nullptr;
    if (cols < 0 || rows < 0 || PyArray_DIM(off, 0) != (npy_intp)cols * rows + 1) {
        PyErr_SetString(PyExc_ValueError, "off must hold cols * rows + 1 offsets");
        return nullptr;
    }
    const int32_t* f = (const int32_t*)PyArray_DATA(flat);
    const int32_t* o = (const int32_t*)PyArray_DATA(off);
    const npy_intp nf = PyArray_DIM(flat, 0);
    for (npy_intp c = 0; c < (npy_intp)cols * rows; ++c)
        if (o[c] < 0 || o[c] > o[c + 1] || o[c + 1] > nf) {
            PyErr_SetString(PyExc_ValueError, "offsets out of order or past the index array");
            return nullptr;
        }
    PyObject* grid = PyList_New(cols);
    if (!grid) return nullptr;
    for (int ix = 0; ix < cols; ++ix) {
        PyObject* col = PyList_New(rows);
        if (!col) {
            Py_DECREF(grid);
            return nullptr;
        }
        PyList_SET_ITEM(grid, ix, col);
        for (int iy = 0; iy < rows; ++iy) {
            const int32_t a = o[ix * rows + iy], b = o[ix * rows + iy + 1];
            PyObject* cell = PyList_New(b - a);
            if (!cell) {
                Py_DECREF(grid);
                return nullptr;
            }
            PyList_SET_ITEM(col, iy, cell);
            for (int32_t j = a; j < b; ++j) {
                PyObject* v = PyLong_FromLong(f[j]);
                if (!v) {
                    Py_DECREF(grid);
                    return nullptr;
                }
                PyList_SET_ITEM(cell, j - a, v);
            }
        }
    }
    return grid;
}

// grid_assign(pts, min_x, min_y, w_inv, h_inv, cols, rows) -> (mGrid, off, flat): Frame.assign_features_to_grid
// + pos_in_grid (Frame.py:143-159) for (n, 2) float64 keypoint coordinates: cell (round((x - min_x) * w_inv),
// round((y - min_y) * h_inv)) in double with round-half-even (Python's round of a float, np.round), keypoints
// outside the grid skipped; mGrid as grid_lists, off / flat the CSR form (int32) the matcher queries.
PyObject* grid_assign(PyObject*, PyObject* args) {
    PyArrayObject* pts;
    double mx, my, wi, hi;
    int cols, rows;
    if (!PyArg_ParseTuple(args, "O!ddddii", &PyArray_Type, &pts, &mx, &my, &wi, &hi, &cols, &rows)) return nullptr;
    if (PyArray_NDIM(pts) != 2 || PyArray_DIM(pts, 1) != 2 || PyArray_TYPE(pts) != NPY_FLOAT64 ||
        !PyArray_IS_C_CONTIGUOUS(pts) || cols <= 0 || rows <= 0) {
        PyErr_SetString(PyExc_ValueError, "pts must be a contiguous (n, 2) float64 array and the grid non-empty");
        return nullptr;
    }
    const npy_intp n = PyArray_DIM(pts, 0), nc = (npy_intp)cols * rows;
    const double* p = (const double*)PyArray_DATA(pts);
    npy_intp dims_off = nc + 1;
    PyArrayObject* off = (PyArrayObject*)PyArray_ZEROS(1, &dims_off, NPY_INT32, 0);
    if (!off) return nullptr;
    int32_t* o = (int32_t*)PyArray_DATA(off);
    int32_t* cell = (int32_t*)PyMem_Malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
    if (!cell) {
        Py_DECREF(off);
        return PyErr_NoMemory();
    }
    npy_intp kept = 0;
    for (npy_intp i = 0; i < n; ++i) {
        const double fx = std::nearbyint((p[2 * i] - mx) * wi), fy = std::nearbyint((p[2 * i + 1] - my) * hi);
        int32_t c = -1;
        if (fx >= 0 && fx < cols && fy >= 0 && fy < rows) {
            c = (int32_t)fx * rows + (int32_t)fy;
            ++o[c + 1];
            ++kept;
        }
        cell[i] = c;
    }
    for (npy_intp c = 0; c < nc; ++c) o[c + 1] += o[c];
    npy_intp dims_flat = kept;
    PyArrayObject* flat = (PyArrayObject*)PyArray_SimpleNew(1, &dims_flat, NPY_INT32);
    if (!flat) {
        PyMem_Free(cell);
        Py_DECREF(off);
        return nullptr;
    }
    int32_t* f = (int32_t*)PyArray_DATA(flat);
    std::vector<int32_t> pos(o, o + nc);  // stable counting sort: keypoint order inside a cell
    for (npy_intp i = 0; i < n; ++i)
        if (cell[i] >= 0) f[pos[cell[i]]++] = (int32_t)i;
    PyMem_Free(cell);
    PyObject* a = Py_BuildValue("(OOii)", (PyObject*)flat, (PyObject*)off, cols, rows);
    PyObject* grid = a ? grid_lists(nullptr, a) : nullptr;
    Py_XDECREF(a);
    if (!grid) {
        Py_DECREF(flat);
        Py_DECREF(off);
        return nullptr;
    }
    return Py_BuildValue("(NNN)", grid, (PyObject*)off, (PyObject*)flat);
}

PyObject* stereo_lists(PyObject*, PyObject* args) {
    PyArrayObject *u, *d, *st, *x;
    double mbf;
    if (!PyArg_ParseTuple(args, "O!O!O!O!d", &PyArray_Type, &u, &PyArray_Type, &d, &PyArray_Type, &st, &PyArray_Type, &x,
                          &mbf) ||
        !contiguous(u, 4, "u") || !contiguous(d, 4, "depth") || !contiguous(st, 1, "status") || !contiguous(x, 4, "x"))
        return nullptr;
    if (PyArray_TYPE(u) != NPY_FLOAT32 || PyArray_TYPE(d) != NPY_FLOAT32 || PyArray_TYPE(x) != NPY_FLOAT32) {
        PyErr_SetString(PyExc_TypeError, "u, depth and x must be float32");
        return nullptr;
    }
    const npy_intp n = PyArray_DIM(u, 0);
    if (PyArray_DIM(d, 0) != n || PyArray_DIM(st, 0) != n || PyArray_DIM(x, 0) < n) {
        PyErr_SetString(PyExc_ValueError, "array lengths differ");
        return nullptr;
    }
    const float* uu = (const float*)PyArray_DATA(u);
    const float* dd = (const float*)PyArray_DATA(d);
    const int8_t* ss = (const int8_t*)PyArray_DATA(st);
    const float* xx = (const float*)PyArray_DATA(x);
    PyArray_Descr* f32 = PyArray_DescrFromType(NPY_FLOAT32);  // new reference
    PyObject* ul = PyList_New(n);
    PyObject* dl = PyList_New(n);
    bool ok = f32 && ul && dl;
    for (npy_intp i = 0; ok && i < n; ++i) {
        PyObject *a, *b;
        if (ss[i] == 1) {
            a = PyArray_Scalar((void*)(uu + i), f32, nullptr);
            b = PyArray_Scalar((void*)(dd + i), f32, nullptr);
        } else if (ss[i] == 2) {
            a = PyFloat_FromDouble((double)xx[i] - 0.01);
            b = PyFloat_FromDouble(mbf / 0.01);
        } else {
            a = PyLong_FromLong(-1);
            b = PyLong_FromLong(-1);
        }
        if (!a || !b) {
            Py_XDECREF(a);
            Py_XDECREF(b);
            ok = false;
            break;
        }
        PyList_SET_ITEM(ul, i, a);
        PyList_SET_ITEM(dl, i, b);
    }
    Py_XDECREF(f32);
    if (!ok) {
        Py_XDECREF(ul);
        Py_XDECREF(dl);
        return PyErr_Occurred() ? nullptr : PyErr_NoMemory();
    }
    return Py_BuildValue("(NN)", ul, dl);
}

PyMethodDef methods[] = {
    {"keypoint_tuples", keypoint_tuples, METH_VARARGS, "cv::KeyPoint tuples of orbfe_keypoint records"},
    {"grid_lists", grid_lists, METH_VARARGS, "Frame.mGrid lists from CSR cell offsets"},
    {"grid_assign", grid_assign, METH_VARARGS, "Frame.assign_features_to_grid: (mGrid, off, flat)"},
    {"stereo_lists", stereo_lists, METH_VARARGS, "Frame.mvuRight / mvDepth lists with the reference's types"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_pyhost", "per-frame Python objects built in C", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__pyhost(void) {
    import_array();
    return PyModule_Create(&module);
}
