"""The JVM boundary's JNI glue, checked without a JDK.

integration/jni/dukehip_jni.c is compiled with -std=c99 -Wall -Wextra -Werror -fsyntax-only
against tests/jni_stub/jni.h, a hand-written jni.h declaring only the JNI types and JNIEnv
functions the glue uses, with the signatures of the JNI specification; and every native
method of DukeHip.java is matched against its C definition: name, return type and the JNI
type of each parameter (Java_io_sesam_dukemicroservice_gpu_DukeHip_<name>(JNIEnv*, jclass,
...)).  The reference side these stand in for: GpuProcessor / GpuBlockingDatabase replace
App.java:329-345 / 450-466.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "integration", "jni", "dukehip_jni.c")
JAVA = os.path.join(ROOT, "integration", "java", "io", "sesam", "dukemicroservice", "gpu", "DukeHip.java")

JNI_TYPE = {"void": "void", "long": "jlong", "int": "jint", "boolean": "jboolean",
            "double": "jdouble", "float": "jfloat", "String": "jstring", "int[]": "jintArray",
            "long[]": "jlongArray", "byte[]": "jbyteArray", "char[]": "jcharArray",
            "double[]": "jdoubleArray", "String[]": "jobjectArray",
            "java.nio.ByteBuffer": "jobject"}


def java_natives():
    src = open(JAVA).read()
    out = {}
    for m in re.finditer(r"static\s+native\s+([\w.\[\]]+)\s+(\w+)\s*\(([^)]*)\)", src, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = []
        for p in params.split(","):
            p = " ".join(p.split())
            if p:
                t = p.rsplit(" ", 1)[0]
                types.append("jobjectArray" if t.endswith("[][]") else JNI_TYPE[t])
        out[name] = (JNI_TYPE[ret], types)
    return out


def c_natives():
    src = open(GLUE).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JFN\((\w+)\)\s*\(([^)]*)\)", src, re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = [" ".join(p.split()) for p in params.split(",")]
        assert ps[0].startswith("JNIEnv* env") and ps[1].startswith("jclass"), name
        out[name] = (ret, [p.rsplit(" ", 1)[0] for p in ps[2:]])
    return out


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_jni_glue_compiles_against_spec_signatures():
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-fsyntax-only", "-I", os.path.join(ROOT, "tests", "jni_stub"),
                        "-I", os.path.join(ROOT, "include"), GLUE],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_java_native_has_a_matching_c_definition():
    j, c = java_natives(), c_natives()
    assert len(j) >= 48
    assert set(j) == set(c), (sorted(set(j) - set(c)), sorted(set(c) - set(j)))
    for name in j:
        assert j[name] == c[name], (name, j[name], c[name])
