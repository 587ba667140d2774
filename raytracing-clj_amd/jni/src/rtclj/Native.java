package rtclj;

/** JNI entry points of librtclj_jni.so (rtclj_jni.c) over include/rt.h. */
public final class Native {
  static {
    System.loadLibrary("rtclj_jni");
  }

  private Native() {}

  /** Linear RGB, rows x width x 3, mean over spp; throws RuntimeException on rt errors. */
  public static native int render(float[] spheres, int[] kinds, float[] mats, float[] camera, int defocus,
                                  int width, int height, int spp, int depth, long seed, int nGpus,
                                  float[] outRgb);

  public static native int deviceCount();
}
