/* _dsyhost: the columns the drop-in host path reads from Python objects, in one C pass each (store_messages, respond).
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
 *
 * SyncCommunity.respond (community.py:2531-2572 in the reference) hands the library, per claim, the four range fields
 * of its ClaimRequest and the 16-byte (record, filter) address pair its BloomFilter keeps (BloomFilter._refs):
 *
 *   claim_columns(requests, ranges, refs) -> None
 *     requests: a list or tuple of ClaimRequests (tuples: time_low, time_high, modulo, offset, bloom, ...);
 *     ranges: writable uint64 buffer of 4 x len(requests); refs: writable buffer of 16 x len(requests) bytes.
 *     A time bound past 2^64 - 1 is stored as 2^63 - 1 (the library clamps every bound there, community.py:2545-2548);
 *     a negative value, or a modulo / offset past 2^64 - 1, raises OverflowError, as numpy's conversion does.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

static PyObject *s_distribution, *s_global_time, *s_packet, *s_meta, *s_refs;

static int get_u64_buffer(PyObject *obj, Py_buffer *view, Py_ssize_t n, const char *name) {
    if (PyObject_GetBuffer(obj, view, PyBUF_WRITABLE | PyBUF_C_CONTIGUOUS) < 0) return -1;
    if (view->len < n * (Py_ssize_t)sizeof(uint64_t)) {
        PyBuffer_Release(view);
        PyErr_Format(PyExc_ValueError, "%s holds fewer than %zd uint64", name, n);
        return -1;
    }
    return 0;
}

/* an integer (int or an __index__ type) as uint64; clamp: a value past 2^64 - 1 becomes 2^63 - 1 instead of raising */
static int as_u64(PyObject *v, int clamp, uint64_t *out) {
    PyObject *i = PyNumber_Index(v);
    if (!i) return -1;
    const unsigned long long x = PyLong_AsUnsignedLongLong(i);
    if (x == (unsigned long long)-1 && PyErr_Occurred()) {
        if (clamp && PyErr_ExceptionMatches(PyExc_OverflowError) && _PyLong_Sign(i) > 0) {
            PyErr_Clear();
            Py_DECREF(i);
            *out = (uint64_t)INT64_MAX;
            return 0;
        }
        Py_DECREF(i);
        return -1;
    }
    Py_DECREF(i);
    *out = (uint64_t)x;
    return 0;
}

static PyObject *claim_columns(PyObject *self, PyObject *args) {
    PyObject *requests, *o_ranges, *o_refs;
    (void)self;
    if (!PyArg_ParseTuple(args, "OOO", &requests, &o_ranges, &o_refs)) return NULL;
    if (!PyList_Check(requests) && !PyTuple_Check(requests)) {
        PyErr_SetString(PyExc_TypeError, "claim_columns: requests must be a list or tuple");
        return NULL;
    }
    /* a tuple snapshot: it holds a reference to every request, so a getter that mutates the caller's list (even
       keeping its length, which may reallocate a list's item array) cannot leave this loop reading freed memory */
    PyObject *seq = PySequence_Tuple(requests);
    if (!seq) return NULL;
    const Py_ssize_t n = PyTuple_GET_SIZE(seq);
    Py_buffer vr, vf;
    if (get_u64_buffer(o_ranges, &vr, 4 * n, "ranges") < 0) {
        Py_DECREF(seq);
        return NULL;
    }
    if (get_u64_buffer(o_refs, &vf, 2 * n, "refs") < 0) {
        PyBuffer_Release(&vr);
        Py_DECREF(seq);
        return NULL;
    }
    uint64_t *ranges = (uint64_t *)vr.buf;
    char *refs = (char *)vf.buf;
    PyObject *ret = NULL;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject *q = PyTuple_GET_ITEM(seq, i);
        if (!PyTuple_Check(q) || PyTuple_GET_SIZE(q) < 5) {
            PyErr_SetString(PyExc_TypeError, "claim_columns: a request is a ClaimRequest tuple");
            goto done;
        }
        int bad = 0;
        for (int f = 0; f < 4 && !bad; ++f) bad = as_u64(PyTuple_GET_ITEM(q, f), f < 2, &ranges[4 * i + f]) < 0;
        PyObject *r = bad ? NULL : PyObject_GetAttr(PyTuple_GET_ITEM(q, 4), s_refs);
        if (!r) goto done;
        if (!PyBytes_Check(r) || PyBytes_GET_SIZE(r) != 16) {
            Py_DECREF(r);
            PyErr_SetString(PyExc_ValueError, "claim_columns: BloomFilter._refs is not 16 bytes");
            goto done;
        }
        memcpy(refs + 16 * i, PyBytes_AS_STRING(r), 16);
        Py_DECREF(r);
    }
    ret = Py_NewRef(Py_None);
done:
    PyBuffer_Release(&vr);
    PyBuffer_Release(&vf);
    Py_DECREF(seq);
    return ret;
}

/* message i's columns (message_columns); 0, or -1 with the exception set */
static int read_message(PyObject *m, Py_ssize_t i, uint64_t *gts, uint64_t *lens, uint64_t *addrs, PyObject *packets,
                        PyObject **first, int *one_meta, int *all_bytes) {
    /* global time: m.distribution.global_time, any integer (int or an __index__ type such as numpy's) */
    PyObject *dist = PyObject_GetAttr(m, s_distribution);
    if (!dist) return -1;
    PyObject *gt = PyObject_GetAttr(dist, s_global_time);
    Py_DECREF(dist);
    if (!gt) return -1;
    PyObject *gti = PyNumber_Index(gt);
    Py_DECREF(gt);
    if (!gti) return -1;
    const unsigned long long g = PyLong_AsUnsignedLongLong(gti);
    Py_DECREF(gti);
    if (g == (unsigned long long)-1 && PyErr_Occurred()) return -1;
    gts[i] = (uint64_t)g;
    /* packet (the list keeps the reference, and with it the bytes the gather list points into) */
    PyObject *p = PyObject_GetAttr(m, s_packet);
    if (!p) return -1;
    PyList_SET_ITEM(packets, i, p); /* steals the reference */
    if (*all_bytes) {
        if (PyBytes_CheckExact(p)) {
            lens[i] = (uint64_t)PyBytes_GET_SIZE(p);
            addrs[i] = (uint64_t)(uintptr_t)PyBytes_AS_STRING(p);
        } else {
            *all_bytes = 0;
        }
    }
    /* meta: getattr(m, "meta", None) compared by identity with the first message's */
    if (*one_meta) {
        PyObject *meta = PyObject_GetAttr(m, s_meta);
        if (!meta) {
            if (!PyErr_ExceptionMatches(PyExc_AttributeError)) return -1;
            PyErr_Clear();
            meta = Py_NewRef(Py_None);
        }
        if (i == 0) {
            *first = meta; /* keeps the reference */
        } else {
            if (meta != *first) *one_meta = 0;
            Py_DECREF(meta);
        }
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
        /* (the getters may run Python code -- properties --: the list must keep its length, and the message is held
           for the duration) */
        if (PyList_GET_SIZE(messages) != n) {
            PyErr_SetString(PyExc_RuntimeError, "message_columns: the message list changed size");
            goto fail;
        }
        PyObject *m = PyList_GET_ITEM(messages, i);
        Py_INCREF(m);
        const int ok = read_message(m, i, gts, lens, addrs, packets, &first, &one_meta, &all_bytes);
        Py_DECREF(m);
        if (ok < 0) goto fail;
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
    {"claim_columns", claim_columns, METH_VARARGS, "claim_columns(requests, ranges, refs) -> None"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_dsyhost", "the drop-in host path's column reads in C (store_messages, respond)", -1,
                                    methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__dsyhost(void) {
    s_distribution = PyUnicode_InternFromString("distribution");
    s_global_time = PyUnicode_InternFromString("global_time");
    s_packet = PyUnicode_InternFromString("packet");
    s_meta = PyUnicode_InternFromString("meta");
    s_refs = PyUnicode_InternFromString("_refs");
    if (!s_distribution || !s_global_time || !s_packet || !s_meta || !s_refs) return NULL;
    return PyModule_Create(&module);
}
