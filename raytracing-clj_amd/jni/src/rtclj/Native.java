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

  /** render with rt_params.flags (RT_FLAG_REALM = 2: the realm.raytracing semantics;
   *  RT_FLAG_REJECTION_SAMPLERS = 8: vec3a's rejection-loop samplers). */
  public static native int renderWithFlags(float[] spheres, int[] kinds, float[] mats, float[] camera,
                                           int defocus, int width, int height, int spp, int depth, long seed,
                                           int nGpus, int flags, float[] outRgb);

  public static final int FLAG_REALM = 2;
  public static final int FLAG_REJECTION_SAMPLERS = 8;

  /** render + write-color! on the device (rt_render_u8): rows x width x 3 bytes. */
  public static native int renderBytes(float[] spheres, int[] kinds, float[] mats, float[] camera, int defocus,
                                       int width, int height, int spp, int depth, long seed, int nGpus, int flags,
                                       byte[] outRgb);

  /** renderBytes without waiting (rt_render_submit_u8): a frame in flight; returns its handle. */
  public static native long submitBytes(float[] spheres, int[] kinds, float[] mats, float[] camera, int defocus,
                                        int width, int height, int spp, int depth, long seed, int nGpus,
                                        int flags);

  /** Waits for a submitted frame (rt_render_wait), copies its bytes into outRgb, frees the handle. */
  public static native int waitBytes(long frame, byte[] outRgb);

  /** -main's camera values (rt_camera_setup) into outCamera[18]; returns the defocus flag. */
  public static native int cameraSetup(int width, int height, double vfov, double[] lookFrom, double[] lookAt,
                                       double[] vup, double defocusAngle, double focusDist, float[] outCamera);

  /** The P3 file of -main (rt_write_ppm). */
  public static native int writePpm(String path, byte[] rgb, int width, int height);

  public static native int deviceCount();

  /** 8-bit RGB PNG of width x height x 3 bytes (rt_write_png). */
  public static native int writePng(String path, byte[] rgb, int width, int height);

  /** ppm2png/ppm->png (src/ppm2png.clj:35-87) through rt_ppm_to_png. */
  public static native int ppmToPng(String srcPpm, String dstPng);
}
