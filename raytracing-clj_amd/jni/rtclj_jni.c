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
 *   static native int renderWithFlags(... the same ..., int nGpus, int flags,
 *                                     float[] outRgb);   // RT_FLAG_REALM: -M:realm
 *   static native int deviceCount();
 *   static native int writePng(String path, byte[] rgb, int width, int height);
 *   static native int ppmToPng(String srcPpm, String dstPng);
 * camera = 18 floats: center, p00, du, dv, disk_u, disk_v (rt_camera order).
 * Replaces compute-pixel + the executor (src/raytracing.clj:141-171) and
 * ppm2png/ppm->png (src/ppm2png.clj:35-87).
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
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

static jint render_impl(JNIEnv* env, jfloatArray spheres, jintArray kinds, jfloatArray mats, jfloatArray camera,
                        jint defocus, jint width, jint height, jint spp, jint depth, jlong seed, jint n_gpus,
                        jint flags, jfloatArray out_rgb) {
  const jsize n = (*env)->GetArrayLength(env, kinds);
  if ((*env)->GetArrayLength(env, spheres) != 4 * n || (*env)->GetArrayLength(env, mats) != 4 * n ||
      (*env)->GetArrayLength(env, camera) != 18) {
    throw_rt(env, RT_E_ARG);
    return RT_E_ARG;
  }
  const jsize out_len = (*env)->GetArrayLength(env, out_rgb);
  /* Copy every input; render into a malloc'd buffer and copy it back with
   * SetFloatArrayRegion.  Nothing is pinned while rt_render runs (a full
   * multi-GPU frame can take seconds: a critical section would block GC
   * JVM-wide for that long). */
  float* sph = (float*)(*env)->GetFloatArrayElements(env, spheres, NULL);
  jint* knd = (*env)->GetIntArrayElements(env, kinds, NULL);
  float* mat = (float*)(*env)->GetFloatArrayElements(env, mats, NULL);
  float* out = (float*)malloc((size_t)out_len * sizeof(float) + 1);
  float cam18[18];
  (*env)->GetFloatArrayRegion(env, camera, 0, 18, cam18);
  int rc = RT_E_ARG;
  if (!sph || !knd || !mat || !out || (*env)->ExceptionCheck(env)) {
    rc = RT_E_ARG; /* an OutOfMemoryError may already be pending */
    goto done;
  }
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
  p.flags = flags;
  rc = rt_render(&scene, &cam, &p, out, (size_t)out_len, NULL);
  if (rc >= 0) (*env)->SetFloatArrayRegion(env, out_rgb, 0, out_len, out);
done:
  free(out);
  if (sph) (*env)->ReleaseFloatArrayElements(env, spheres, (jfloat*)sph, JNI_ABORT);
  if (knd) (*env)->ReleaseIntArrayElements(env, kinds, knd, JNI_ABORT);
  if (mat) (*env)->ReleaseFloatArrayElements(env, mats, (jfloat*)mat, JNI_ABORT);
  if (rc < 0 && !(*env)->ExceptionCheck(env)) throw_rt(env, rc);
  return rc;
}

JNIEXPORT jint JNICALL Java_rtclj_Native_render(JNIEnv* env, jclass cls, jfloatArray spheres, jintArray kinds,
                                                jfloatArray mats, jfloatArray camera, jint defocus, jint width,
                                                jint height, jint spp, jint depth, jlong seed, jint n_gpus,
                                                jfloatArray out_rgb) {
  (void)cls;
  return render_impl(env, spheres, kinds, mats, camera, defocus, width, height, spp, depth, seed, n_gpus, 0,
                     out_rgb);
}

JNIEXPORT jint JNICALL Java_rtclj_Native_renderWithFlags(JNIEnv* env, jclass cls, jfloatArray spheres,
                                                         jintArray kinds, jfloatArray mats, jfloatArray camera,
                                                         jint defocus, jint width, jint height, jint spp,
                                                         jint depth, jlong seed, jint n_gpus, jint flags,
                                                         jfloatArray out_rgb) {
  (void)cls;
  return render_impl(env, spheres, kinds, mats, camera, defocus, width, height, spp, depth, seed, n_gpus, flags,
                     out_rgb);
}

JNIEXPORT jint JNICALL Java_rtclj_Native_writePng(JNIEnv* env, jclass cls, jstring path, jbyteArray rgb, jint width,
                                                  jint height) {
  (void)cls;
  if ((jlong)(*env)->GetArrayLength(env, rgb) < (jlong)width * height * 3) {
    throw_rt(env, RT_E_ARG);
    return RT_E_ARG;
  }
  const char* p = (*env)->GetStringUTFChars(env, path, NULL);
  jbyte* px = (*env)->GetByteArrayElements(env, rgb, NULL);
  const int rc = (p && px) ? rt_write_png(p, (const uint8_t*)px, width, height) : RT_E_ARG;
  if (px) (*env)->ReleaseByteArrayElements(env, rgb, px, JNI_ABORT);
  if (p) (*env)->ReleaseStringUTFChars(env, path, p);
  if (rc < 0) throw_rt(env, rc);
  return rc;
}

JNIEXPORT jint JNICALL Java_rtclj_Native_ppmToPng(JNIEnv* env, jclass cls, jstring src, jstring dst) {
  (void)cls;
  const char* s = (*env)->GetStringUTFChars(env, src, NULL);
  const char* d = (*env)->GetStringUTFChars(env, dst, NULL);
  const int rc = (s && d) ? rt_ppm_to_png(s, d) : RT_E_ARG;
  if (d) (*env)->ReleaseStringUTFChars(env, dst, d);
  if (s) (*env)->ReleaseStringUTFChars(env, src, s);
  if (rc < 0) throw_rt(env, rc);
  return rc;
}
