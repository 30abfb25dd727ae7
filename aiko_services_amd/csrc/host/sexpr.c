/* Native S-expression codec: the control plane's wire format (aiko_services_amd/utils/sexpr.py).
 *
 * Every actor message and every process_frame / process_frame_response metadata record passes
 * through parse() and generate(); at thousands of hop messages per second on a pipeline-parallel
 * rank 0 the per-character Python scanner was the largest single cost of the control plane.
 * This module implements the same grammar (reference codec:
 * /root/reference/src/aiko_services/main/utilities/parser.py:85-227) in one pass over the UTF-8
 * / UCS buffer:
 *
 *   scan(payload)   -> nested lists of str / None (the raw tree, sexpr._Scanner semantics)
 *   to_dict(tree)   -> sexpr.parse_list_to_dict(tree)  (a list whose car is "key:" -> dict)
 *   generate(expr)  -> sexpr.generate_s_expression(expr)
 *
 * Semantics match the Python implementation exactly (tests/test_sexpr_native.py fuzzes both).
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

/* ---- scan ------------------------------------------------------------------------------------ */

typedef struct {
    int kind;
    const void *data;
    Py_ssize_t n;
    Py_ssize_t i;
    PyObject *src;
} Scanner;

#define CH(sc, k) PyUnicode_READ((sc)->kind, (sc)->data, (k))

static inline int is_ws(Py_UCS4 c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

static int append_token(PyObject *list, Scanner *sc, Py_ssize_t a, Py_ssize_t b) {
    PyObject *t = PyUnicode_Substring(sc->src, a, b);
    if (!t) return -1;
    int r = PyList_Append(list, t);
    Py_DECREF(t);
    return r;
}

/* canonical "digits:data" at token start: 1 = consumed (token appended), 0 = not canonical */
static int try_canonical(Scanner *sc, PyObject *list) {
    Py_ssize_t i = sc->i, j = i, n = sc->n;
    while (j < n) {
        Py_UCS4 c = CH(sc, j);
        if (c < '0' || c > '9') break;
        j++;
    }
    if (j == i || j >= n || CH(sc, j) != ':' || j + 1 >= n) return 0;
    Py_ssize_t length = 0;
    for (Py_ssize_t k = i; k < j; k++) {
        length = length * 10 + (Py_ssize_t)(CH(sc, k) - '0');
        if (length > n) { length = n + 1; }          /* saturate: the slice is clipped anyway */
    }
    Py_ssize_t start = j + 1;
    if (length == 0) {
        sc->i = start;
        return PyList_Append(list, Py_None) < 0 ? -1 : 1;
    }
    Py_ssize_t end = start + length;
    sc->i = end;
    if (end > n) end = n;
    return append_token(list, sc, start, end) < 0 ? -1 : 1;
}

static int try_quoted(Scanner *sc, PyObject *list) {
    Py_UCS4 q = CH(sc, sc->i);
    if (q != '"' && q != '\'') return 0;
    Py_ssize_t end = PyUnicode_FindChar(sc->src, q, sc->i + 1, sc->n, 1);
    if (end == -2) return -1;
    if (end < 0) return 0;
    Py_ssize_t a = sc->i + 1;
    sc->i = end + 1;
    return append_token(list, sc, a, end) < 0 ? -1 : 1;
}

static PyObject *scan_list(Scanner *sc, int depth) {
    if (depth > 512) {
        PyErr_SetString(PyExc_ValueError, "S-Expression nested too deeply");
        return NULL;
    }
    PyObject *result = PyList_New(0);
    if (!result) return NULL;
    Py_ssize_t token_start = -1;
    while (sc->i < sc->n) {
        if (token_start < 0) {
            int r = try_canonical(sc, result);
            if (r < 0) goto fail;
            if (r) continue;
            r = try_quoted(sc, result);
            if (r < 0) goto fail;
            if (r) continue;
        }
        Py_UCS4 c = CH(sc, sc->i);
        if (c == '(') {
            if (token_start >= 0) {
                if (append_token(result, sc, token_start, sc->i) < 0) goto fail;
                token_start = -1;
            }
            sc->i++;
            PyObject *sub = scan_list(sc, depth + 1);
            if (!sub) goto fail;
            int r = PyList_Append(result, sub);
            Py_DECREF(sub);
            if (r < 0) goto fail;
            continue;
        }
        if (c == ')') {
            if (token_start >= 0 && append_token(result, sc, token_start, sc->i) < 0) goto fail;
            sc->i++;
            return result;
        }
        if (is_ws(c)) {
            if (token_start >= 0) {
                if (append_token(result, sc, token_start, sc->i) < 0) goto fail;
                token_start = -1;
            }
        } else if (token_start < 0) {
            token_start = sc->i;
        }
        sc->i++;
    }
    if (token_start >= 0 && append_token(result, sc, token_start, sc->n) < 0) goto fail;
    return result;
fail:
    Py_DECREF(result);
    return NULL;
}

static PyObject *py_scan(PyObject *self, PyObject *arg) {
    (void)self;
    if (!PyUnicode_Check(arg)) {
        PyErr_SetString(PyExc_TypeError, "scan() expects str");
        return NULL;
    }
    if (PyUnicode_READY(arg) < 0) return NULL;
    Scanner sc = {PyUnicode_KIND(arg), PyUnicode_DATA(arg), PyUnicode_GET_LENGTH(arg), 0, arg};
    return scan_list(&sc, 0);
}

/* ---- to_dict --------------------------------------------------------------------------------- */

static int ends_with_colon(PyObject *s) {
    Py_ssize_t n = PyUnicode_GET_LENGTH(s);
    return n > 0 && PyUnicode_READ_CHAR(s, n - 1) == ':';
}

static PyObject *to_dict(PyObject *tree, int depth) {
    if (!PyList_Check(tree) || PyList_GET_SIZE(tree) == 0) {
        Py_INCREF(tree);
        return tree;
    }
    if (depth > 512) {
        PyErr_SetString(PyExc_ValueError, "S-Expression nested too deeply");
        return NULL;
    }
    Py_ssize_t n = PyList_GET_SIZE(tree);
    PyObject *car = PyList_GET_ITEM(tree, 0);
    if (PyUnicode_Check(car) && ends_with_colon(car)) {
        if (n % 2) {
            PyErr_Format(PyExc_ValueError,
                         "Error parsing S-Expression dictionary starting at keyword \"%U\", "
                         "must have pairs of keywords and values", car);
            return NULL;
        }
        PyObject *out = PyDict_New();
        if (!out) return NULL;
        for (Py_ssize_t i = 0; i < n; i += 2) {
            PyObject *key = PyList_GET_ITEM(tree, i);
            if (!PyUnicode_Check(key)) {
                PyObject *r = PyObject_Str(key);
                PyErr_Format(PyExc_ValueError,
                             "Error parsing S-Expression dictionary starting at keyword \"%U\", "
                             "keyword must be a string", r ? r : Py_None);
                Py_XDECREF(r);
                Py_DECREF(out);
                return NULL;
            }
            Py_ssize_t kn = PyUnicode_GET_LENGTH(key);
            if (kn && !ends_with_colon(key)) {
                PyErr_Format(PyExc_ValueError,
                             "Error parsing S-Expression dictionary starting at keyword \"%U\", "
                             "keyword must end with \":\" character", key);
                Py_DECREF(out);
                return NULL;
            }
            PyObject *k = PyUnicode_Substring(key, 0, kn ? kn - 1 : 0);
            PyObject *v = k ? to_dict(PyList_GET_ITEM(tree, i + 1), depth + 1) : NULL;
            if (!v || PyDict_SetItem(out, k, v) < 0) {
                Py_XDECREF(k);
                Py_XDECREF(v);
                Py_DECREF(out);
                return NULL;
            }
            Py_DECREF(k);
            Py_DECREF(v);
        }
        return out;
    }
    PyObject *out = PyList_New(n);
    if (!out) return NULL;
    for (Py_ssize_t i = 0; i < n; i++) {
        PyObject *v = to_dict(PyList_GET_ITEM(tree, i), depth + 1);
        if (!v) {
            Py_DECREF(out);
            return NULL;
        }
        PyList_SET_ITEM(out, i, v);
    }
    return out;
}

static PyObject *py_to_dict(PyObject *self, PyObject *arg) {
    (void)self;
    return to_dict(arg, 0);
}

/* ---- generate -------------------------------------------------------------------------------- */

typedef struct {
    _PyUnicodeWriter w;
} Gen;

static int needs_canonical(PyObject *s) {
    Py_ssize_t n = PyUnicode_GET_LENGTH(s);
    if (n == 0) return 0;
    int kind = PyUnicode_KIND(s);
    const void *d = PyUnicode_DATA(s);
    for (Py_ssize_t k = 0; k < n; k++) {
        Py_UCS4 c = PyUnicode_READ(kind, d, k);
        if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '(' || c == ')') return 1;
    }
    /* leading "digits:" would be mistaken for a canonical length prefix (str.isdigit: ASCII
       and other Unicode decimal digits) */
    Py_ssize_t i = 0;
    while (i < n && Py_UNICODE_ISDIGIT(PyUnicode_READ(kind, d, i))) i++;
    return i > 0 && i < n && PyUnicode_READ(kind, d, i) == ':';
}

static int gen_expr(Gen *g, PyObject *expr, int depth, int pairs);

static int gen_scalar(Gen *g, PyObject *el, int depth) {
    if (el == Py_None) return _PyUnicodeWriter_WriteASCIIString(&g->w, "0:", 2);
    if (PyUnicode_Check(el)) {
        Py_ssize_t n = PyUnicode_GET_LENGTH(el);
        if (n == 0) return _PyUnicodeWriter_WriteASCIIString(&g->w, "\"\"", 2);
        if (needs_canonical(el)) {
            char buf[32];
            int m = snprintf(buf, sizeof buf, "%zd:", n);
            if (_PyUnicodeWriter_WriteASCIIString(&g->w, buf, m) < 0) return -1;
        }
        return _PyUnicodeWriter_WriteStr(&g->w, el);
    }
    if (PyDict_Check(el) || PyList_Check(el) || PyTuple_Check(el)) return gen_expr(g, el, depth + 1, 1);
    /* arrays never become text (str(tensor) is lossy and unparseable): the caller sends them with
       message/tensor_payload.py; same rule as sexpr.py _refuse_array */
    if (!PyLong_Check(el) && !PyFloat_Check(el) &&
        (PyObject_HasAttrString(el, "__dlpack__") || PyObject_HasAttrString(el, "__array_interface__") ||
         PyObject_HasAttrString((PyObject *)Py_TYPE(el), "__aiko_device_result__"))) {
        PyErr_Format(PyExc_TypeError,
                     "generate(): cannot render %s as an S-expression (use message.tensor_payload.encode_message)",
                     Py_TYPE(el)->tp_name);
        return -1;
    }
    PyObject *s = PyObject_Str(el);
    if (!s) return -1;
    int r = _PyUnicodeWriter_WriteStr(&g->w, s);
    Py_DECREF(s);
    return r;
}

/* pairs: a dict renders as its key: value pairs (nested values); a top-level dict iterates its
   keys, as the Python generator does */
static int gen_expr(Gen *g, PyObject *expr, int depth, int pairs) {
    if (depth > 512) {
        PyErr_SetString(PyExc_ValueError, "S-Expression nested too deeply");
        return -1;
    }
    if (_PyUnicodeWriter_WriteChar(&g->w, '(') < 0) return -1;
    int first = 1;
    if (pairs && PyDict_Check(expr)) {
        PyObject *k, *v;
        Py_ssize_t pos = 0;
        while (PyDict_Next(expr, &pos, &k, &v)) {
            if (!first && _PyUnicodeWriter_WriteChar(&g->w, ' ') < 0) return -1;
            first = 0;
            /* f"{k}:" is a str: emitted as-is when it needs no canonical form */
            PyObject *ks = PyUnicode_Check(k) ? (Py_INCREF(k), k) : PyObject_Str(k);
            if (!ks) return -1;
            PyObject *key = PyUnicode_FromFormat("%U:", ks);
            Py_DECREF(ks);
            if (!key) return -1;
            int r = gen_scalar(g, key, depth);
            Py_DECREF(key);
            if (r < 0) return -1;
            if (_PyUnicodeWriter_WriteChar(&g->w, ' ') < 0) return -1;
            if (gen_scalar(g, v, depth) < 0) return -1;
        }
    } else {
        PyObject *seq = PySequence_Fast(expr, "generate() expects a list, tuple or dict");
        if (!seq) return -1;
        Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
        PyObject **items = PySequence_Fast_ITEMS(seq);
        for (Py_ssize_t i = 0; i < n; i++) {
            if (!first && _PyUnicodeWriter_WriteChar(&g->w, ' ') < 0) {
                Py_DECREF(seq);
                return -1;
            }
            first = 0;
            if (gen_scalar(g, items[i], depth) < 0) {
                Py_DECREF(seq);
                return -1;
            }
        }
        Py_DECREF(seq);
    }
    return _PyUnicodeWriter_WriteChar(&g->w, ')');
}

static PyObject *py_generate(PyObject *self, PyObject *arg) {
    (void)self;
    Gen g;
    _PyUnicodeWriter_Init(&g.w);
    g.w.overallocate = 1;
    if (gen_expr(&g, arg, 0, 0) < 0) {
        _PyUnicodeWriter_Dealloc(&g.w);
        return NULL;
    }
    return _PyUnicodeWriter_Finish(&g.w);
}

static PyMethodDef methods[] = {
    {"scan", py_scan, METH_O, "Raw S-expression tree of a payload (lists of str / None)."},
    {"to_dict", py_to_dict, METH_O, "Lists whose first element is a 'key:' symbol become dicts."},
    {"generate", py_generate, METH_O, "S-expression text of a list / tuple / dict."},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_sexpr", "Native S-expression codec.", -1, methods};

PyMODINIT_FUNC PyInit__sexpr(void) { return PyModule_Create(&module); }
