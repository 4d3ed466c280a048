/* _dsyhost: the columns SyncCommunity.store_messages reads from a batch of received messages, in one C pass.
 *
 * Dispersy._store (dispersy.py:1475-1533) walks its messages one by one for the INSERT's values: the packet, the
 * distribution's global time and the meta's database id.  The Python mirror (dispersy_amd/community.py
 * store_messages) reads them column by column with C-level getters; this module reads all of them in one pass over
 * the list and hands SyncStore.append the gather list (packet addresses and lengths) dsy_store_append_gather takes,
 * so no per-message Python frame or intermediate list is built.  Host code only (no GPU, no HIP); the results are
 * exactly the Python path's (tests/test_sequence.py checks both on the same batches).
 *
 *   message_columns(messages, gts, lens, addrs) -> (packets, one_meta, first_meta, all_bytes)
 *     messages: a list; gts, lens, addrs: writable C-contiguous buffers of len(messages) uint64 each.
 *     gts[i]   = messages[i].distribution.global_time (an integer, as the INSERT's global_time)
 *     lens[i]  = len(messages[i].packet), addrs[i] = the address of its bytes -- filled while every packet is exactly
 *                bytes; all_bytes says whether they all were (else the caller takes its byte-joining path)
 *     packets  = [m.packet for m in messages] (new list, the packets' references: they keep the bytes alive)
 *     one_meta = every message's .meta (None when it has none) is the first message's object; first_meta = that.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

static PyObject *s_distribution, *s_global_time, *s_packet, *s_meta;

static int get_u64_buffer(PyObject *obj, Py_buffer *view, Py_ssize_t n, const char *name) {
    if (PyObject_GetBuffer(obj, view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) return -1;
    if (view->len < n * (Py_ssize_t)sizeof(uint64_t)) {
        PyBuffer_Release(view);
        PyErr_Format(PyExc_ValueError, "message_columns: %s holds fewer than %zd uint64", name, n);
        return -1;
    }
    return 0;
}

static PyObject *message_columns(PyObject *self, PyObject *args) {
    PyObject *messages, *o_gts, *o_lens, *o_addrs;
    (void)self;
    if (!PyArg_ParseTuple(args, "O!OOO", &PyList_Type, &messages, &o_gts, &o_lens, &o_addrs)) return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(messages);
    Py_buffer vg, vl, va;
    if (get_u64_buffer(o_gts, &vg, n, "gts") < 0) return NULL;
    if (get_u64_buffer(o_lens, &vl, n, "lens") < 0) {
        PyBuffer_Release(&vg);
        return NULL;
    }
    if (get_u64_buffer(o_addrs, &va, n, "addrs") < 0) {
        PyBuffer_Release(&vg);
        PyBuffer_Release(&vl);
        return NULL;
    }
    uint64_t *gts = (uint64_t *)vg.buf, *lens = (uint64_t *)vl.buf, *addrs = (uint64_t *)va.buf;
    PyObject *packets = PyList_New(n), *first = NULL, *result = NULL;
    int one_meta = 1, all_bytes = 1;
    if (!packets) goto done;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *m = PyList_GET_ITEM(messages, i);
        /* global time: m.distribution.global_time, any integer (int or an __index__ type such as numpy's) */
        PyObject *dist = PyObject_GetAttr(m, s_distribution);
        if (!dist) goto fail;
        PyObject *gt = PyObject_GetAttr(dist, s_global_time);
        Py_DECREF(dist);
        if (!gt) goto fail;
        PyObject *gti = PyNumber_Index(gt);
        Py_DECREF(gt);
        if (!gti) goto fail;
        const unsigned long long g = PyLong_AsUnsignedLongLong(gti);
        Py_DECREF(gti);
        if (g == (unsigned long long)-1 && PyErr_Occurred()) goto fail;
        gts[i] = (uint64_t)g;
        /* packet */
        PyObject *p = PyObject_GetAttr(m, s_packet);
        if (!p) goto fail;
        PyList_SET_ITEM(packets, i, p); /* steals the reference */
        if (all_bytes) {
            if (PyBytes_CheckExact(p)) {
                lens[i] = (uint64_t)PyBytes_GET_SIZE(p);
                addrs[i] = (uint64_t)(uintptr_t)PyBytes_AS_STRING(p);
            } else {
                all_bytes = 0;
            }
        }
        /* meta: getattr(m, "meta", None) compared by identity with the first message's */
        if (one_meta) {
            PyObject *meta = PyObject_GetAttr(m, s_meta);
            if (!meta) {
                if (!PyErr_ExceptionMatches(PyExc_AttributeError)) goto fail;
                PyErr_Clear();
                meta = Py_None;
                Py_INCREF(meta);
            }
            if (i == 0) {
                first = meta; /* keeps the reference */
            } else {
                if (meta != first) one_meta = 0;
                Py_DECREF(meta);
            }
        }
    }
    if (!first) {
        first = Py_None;
        Py_INCREF(first);
    }
    result = Py_BuildValue("(NNNN)", packets, PyBool_FromLong(one_meta), one_meta ? first : Py_NewRef(Py_None),
                           PyBool_FromLong(all_bytes));
    packets = NULL;
    if (one_meta) first = NULL; /* its reference went into the tuple */
    goto done;
fail:
    Py_CLEAR(packets);
done:
    Py_XDECREF(first);
    PyBuffer_Release(&vg);
    PyBuffer_Release(&vl);
    PyBuffer_Release(&va);
    return result;
}

static PyMethodDef methods[] = {
    {"message_columns", message_columns, METH_VARARGS,
     "message_columns(messages, gts, lens, addrs) -> (packets, one_meta, first_meta, all_bytes)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dsyhost", "store_messages' column reads in C", -1,
                                    methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__dsyhost(void) {
    s_distribution = PyUnicode_InternFromString("distribution");
    s_global_time = PyUnicode_InternFromString("global_time");
    s_packet = PyUnicode_InternFromString("packet");
    s_meta = PyUnicode_InternFromString("meta");
    if (!s_distribution || !s_global_time || !s_packet || !s_meta) return NULL;
    return PyModule_Create(&module);
}
