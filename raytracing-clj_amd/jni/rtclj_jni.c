/*
 * rtclj_jni.c — JNI shim binding the Clojure host (keychera/raytracing-clj)
 * to include/rt.h.  Built only where a JDK exists (`make -C raytracing-clj_amd
 * jni JAVA_HOME=...`); this image has no jni.h, so it is not compiled here.
 *
 * Java side: class rtclj.Native
 *   static native int render(float[] spheres, int[] kinds, float[] mats,
 *                            float[] camera, int defocus, int width, int height,
 *                            int spp, int depth, long seed, int nGpus,
 *                            float[] outRgb);
 *   static native int deviceCount();
 * camera = 18 floats: center, p00, du, dv, disk_u, disk_v (rt_camera order).
 * Replaces compute-pixel + the executor (src/raytracing.clj:141-171).
 */
#include <jni.h>
#include <stdio.h>
#include <string.h>

#include "../../include/rt.h"

static void throw_rt(JNIEnv* env, int code) {
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  if (ex) {
    char msg[512];
    snprintf(msg, sizeof msg, "rt error %d: %s", code, rt_last_error());
    (*env)->ThrowNew(env, ex, msg);
  }
}

JNIEXPORT jint JNICALL Java_rtclj_Native_deviceCount(JNIEnv* env, jclass cls) {
  (void)env;
  (void)cls;
  return rt_device_count();
}

JNIEXPORT jint JNICALL Java_rtclj_Native_render(JNIEnv* env, jclass cls, jfloatArray spheres, jintArray kinds,
                                                jfloatArray mats, jfloatArray camera, jint defocus, jint width,
                                                jint height, jint spp, jint depth, jlong seed, jint n_gpus,
                                                jfloatArray out_rgb) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, kinds);
  if ((*env)->GetArrayLength(env, spheres) != 4 * n || (*env)->GetArrayLength(env, mats) != 4 * n ||
      (*env)->GetArrayLength(env, camera) != 18) {
    throw_rt(env, RT_E_ARG);
    return RT_E_ARG;
  }
  const jsize out_len = (*env)->GetArrayLength(env, out_rgb);
  /* copy the small inputs; pin only the framebuffer (no JNI calls while it is pinned) */
  float* sph = (float*)(*env)->GetFloatArrayElements(env, spheres, NULL);
  jint* knd = (*env)->GetIntArrayElements(env, kinds, NULL);
  float* mat = (float*)(*env)->GetFloatArrayElements(env, mats, NULL);
  float cam18[18];
  (*env)->GetFloatArrayRegion(env, camera, 0, 18, cam18);
  rt_camera cam;
  memcpy(cam.center, cam18 + 0, 12);
  memcpy(cam.p00, cam18 + 3, 12);
  memcpy(cam.du, cam18 + 6, 12);
  memcpy(cam.dv, cam18 + 9, 12);
  memcpy(cam.disk_u, cam18 + 12, 12);
  memcpy(cam.disk_v, cam18 + 15, 12);
  cam.defocus = defocus;
  rt_scene scene = {(int)n, sph, (const int*)knd, mat};
  rt_params p;
  memset(&p, 0, sizeof p);
  p.width = width;
  p.height = height;
  p.row_begin = 0;
  p.row_end = height;
  p.spp = spp;
  p.max_depth = depth;
  p.seed = (uint64_t)seed;
  p.n_devices = n_gpus;
  float* out = (float*)(*env)->GetPrimitiveArrayCritical(env, out_rgb, NULL);
  const int rc = rt_render(&scene, &cam, &p, out, (size_t)out_len, NULL);
  (*env)->ReleasePrimitiveArrayCritical(env, out_rgb, out, 0);
  (*env)->ReleaseFloatArrayElements(env, spheres, (jfloat*)sph, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, kinds, knd, JNI_ABORT);
  (*env)->ReleaseFloatArrayElements(env, mats, (jfloat*)mat, JNI_ABORT);
  if (rc < 0) throw_rt(env, rc);
  return rc;
}
