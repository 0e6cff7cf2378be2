"""The Kotlin drop-in as source (barnes-hut-n-body_amd/kotlin/): the `external fun`s of
Native.kt must be exactly the natives barnes-hut-n-body_amd/jni/bh_jni.c exports, with JNI
signatures that match (there is no JDK here to compile either side against the other), and
PhysicsEngine.kt must offer the reference surface NBodyPanel.kt calls (BarnesHutAlg.kt:287-349:
the constructor, step, getBodies, resetBodies, getTreeForDebug().visitQuads, mergeMaxMass,
mergeMinDist)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KT = os.path.join(ROOT, "barnes-hut-n-body_amd", "kotlin")
JNI_C = os.path.join(ROOT, "barnes-hut-n-body_amd", "jni", "bh_jni.c")

# Kotlin parameter / return types -> the JNI C types javac -h would emit
KT2JNI = {"Int": "jint", "Long": "jlong", "Double": "jdouble", "DoubleArray": "jdoubleArray",
          "IntArray": "jintArray", "LongArray": "jlongArray", "ByteBuffer": "jobject",
          "Unit": "void"}


def kotlin_externals():
    src = open(os.path.join(KT, "Native.kt")).read()
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"external\s+fun\s+(\w+)\s*\(([^)]*)\)\s*(?::\s*(\w+))?", src):
        name, params, ret = m.group(1), m.group(2), m.group(3) or "Unit"
        types = [p.split(":")[1].strip() for p in params.split(",") if p.strip()]
        out[name] = ([KT2JNI[t] for t in types], KT2JNI[ret])
    return out


def jni_exports():
    src = open(JNI_C).read()
    out = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+Java_Native_(\w+)\s*\(([^)]*)\)", src,
                         flags=re.S):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = [" ".join(p.split()[:-1]).replace("*", "").strip() for p in params.split(",")]
        assert types[:2] == ["JNIEnv", "jobject"], (name, types)  # (env, the object's `this`)
        out[name] = (types[2:], ret)
    return out


def test_native_externals_match_the_jni_exports():
    kt, c = kotlin_externals(), jni_exports()
    assert set(kt) == set(c), f"Kotlin {sorted(kt)} vs C {sorted(c)}"
    for name in kt:
        assert kt[name] == c[name], f"{name}: Kotlin {kt[name]} vs C {c[name]}"
    assert len(kt) == 13


def test_physics_engine_offers_the_reference_surface():
    src = open(os.path.join(KT, "PhysicsEngine.kt")).read()
    assert re.search(r"class\s+PhysicsEngine\s*\(\s*initialBodies\s*:\s*MutableList<Body>\s*\)", src)
    for sig in (r"fun\s+step\s*\(\s*\)", r"fun\s+getBodies\s*\(\s*\)\s*:\s*List<Body>",
                r"fun\s+resetBodies\s*\(\s*newBodies\s*:\s*MutableList<Body>\s*\)",
                r"fun\s+getTreeForDebug\s*\(\s*\)", r"var\s+mergeMaxMass\s*:\s*Double",
                r"var\s+mergeMinDist\s*:\s*Double",
                r"fun\s+visitQuads\s*\(\s*visit\s*:\s*\(Quad\)\s*->\s*Unit\s*\)"):
        assert re.search(sig, src), sig
    # every native it calls is declared
    code = re.sub(r"//[^\n]*", "", src)
    used = set(re.findall(r"Native\.(\w+)\s*\(", code))
    assert used <= set(kotlin_externals()), used - set(kotlin_externals())
