(ns raytracing.gpu
  "Drop-in GPU path for the reference's -main (src/raytracing.clj:95-177):
  scene, camera and PPM stay in Clojure; compute-pixel + the executor
  (raytracing.clj:141-171) become one call into the MI355X kernel through
  rtclj.Native (JNI -> include/rt.h rt_render).  Bodies carry their
  parameters as data, because the reference's closures hide them."
  (:import [rtclj Native]))

(def kind {:lambertian 0 :metal 1 :dielectric 2 nil 3})

(defn flatten-bodies
  "[{:center [x y z] :radius r :material {:type :metal :albedo [r g b] :fuzz f}} ...]
  -> [spheres kinds mats] primitive arrays in rt_scene layout."
  [bodies]
  (let [n (count bodies)
        sph (float-array (* 4 n))
        knd (int-array n)
        mat (float-array (* 4 n))]
    (doseq [[i {:keys [center radius material]}] (map-indexed vector bodies)]
      (let [[x y z] center
            [r g b] (:albedo material [0 0 0])]
        (aset sph (* 4 i) (float x))
        (aset sph (+ 1 (* 4 i)) (float y))
        (aset sph (+ 2 (* 4 i)) (float z))
        (aset sph (+ 3 (* 4 i)) (float radius))
        (aset knd i (int (kind (:type material))))
        (aset mat (* 4 i) (float r))
        (aset mat (+ 1 (* 4 i)) (float g))
        (aset mat (+ 2 (* 4 i)) (float b))
        (aset mat (+ 3 (* 4 i)) (float (or (:fuzz material) (:refraction-index material) 0.0)))))
    [sph knd mat]))

(defn- flags
  "rt_params.flags of an options map: :realm? (RT_FLAG_REALM) and
  :rejection-samplers? (RT_FLAG_REJECTION_SAMPLERS: vec3a's own rejection
  loops instead of the kernel's loop-free samplers of the same distributions)."
  [{:keys [realm? rejection-samplers?]}]
  (bit-or (if realm? Native/FLAG_REALM 0) (if rejection-samplers? Native/FLAG_REJECTION_SAMPLERS 0)))

(defn render
  "width*height*3 linear RGB floats: compute-pixel's accum/spp for every pixel.
  camera keys are the values -main derives (raytracing.clj:126-139).
  :realm? true renders with realm.raytracing's semantics (RT_FLAG_REALM:
  src/realm/raytracing.clj; pass realm's camera: no defocus, focal length
  |look-from - look-at|).  :rejection-samplers? true draws vec3a's
  random-unit-vec3 / random-in-unit-disk by their rejection loops
  (RT_FLAG_REJECTION_SAMPLERS); the default draws the same distributions
  loop-free."
  [bodies {:keys [center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v defocus-angle]}
   {:keys [width height samples-per-px max-depth seed gpus] :or {seed 1 gpus 0} :as opts}]
  (let [[sph knd mat] (flatten-bodies bodies)
        cam (float-array (concat center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v))
        out (float-array (* width height 3))]
    (Native/renderWithFlags sph knd mat cam (if (pos? (or defocus-angle 0)) 1 0) width height
                            samples-per-px max-depth (long seed) (int gpus)
                            (flags opts) out)
    out))

(defn render-bytes
  "render, then write-color! on the device (rt_render_u8): width*height*3
  bytes, the 0..255 values -main writes (raytracing.clj:19-26)."
  [bodies {:keys [center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v defocus-angle]}
   {:keys [width height samples-per-px max-depth seed gpus] :or {seed 1 gpus 0} :as opts}]
  (let [[sph knd mat] (flatten-bodies bodies)
        cam (float-array (concat center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v))
        out (byte-array (* width height 3))]
    (Native/renderBytes sph knd mat cam (if (pos? (or defocus-angle 0)) 1 0) width height
                        samples-per-px max-depth (long seed) (int gpus)
                        (flags opts) out)
    out))

(defn submit-bytes
  "render-bytes without waiting (rt_render_submit_u8): returns a frame in
  flight for await-bytes.  A host drawing a sequence of frames submits the
  next before it awaits the last, as the executor's futures do
  (raytracing.clj:157-171)."
  [bodies {:keys [center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v defocus-angle]}
   {:keys [width height samples-per-px max-depth seed gpus] :or {seed 1 gpus 0} :as opts}]
  (let [[sph knd mat] (flatten-bodies bodies)
        cam (float-array (concat center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v))]
    {:handle (Native/submitBytes sph knd mat cam (if (pos? (or defocus-angle 0)) 1 0) width height
                                 samples-per-px max-depth (long seed) (int gpus)
                                 (flags opts))
     :size (* width height 3)}))

(defn await-bytes
  "The bytes of a frame from submit-bytes (rt_render_wait); each frame is
  awaited exactly once."
  [{:keys [handle size]}]
  (let [out (byte-array size)]
    (Native/waitBytes handle out)
    out))

(defn camera
  "-main's camera values (raytracing.clj:105-139) through rt_camera_setup, in
  the keys render takes."
  [width height {:keys [vfov look-from look-at vup defocus-angle focus-dist]}]
  (let [out (float-array 18)
        _ (Native/cameraSetup (int width) (int height) (double vfov) (double-array look-from)
                              (double-array look-at) (double-array vup) (double defocus-angle)
                              (double focus-dist) out)
        v (fn [i] (vec (take 3 (drop i out))))]
    {:center (v 0) :pixel-00-loc (v 3) :pixel-du (v 6) :pixel-dv (v 9)
     :defocus-disk-u (v 12) :defocus-disk-v (v 15) :defocus-angle defocus-angle}))

(defn write-ppm!
  "rgb: width*height*3 bytes -> the P3 file -main writes (raytracing.clj:172-175)."
  [path ^bytes rgb width height]
  (Native/writePpm (str path) rgb (int width) (int height)))

(defn write-png!
  "rgb: width*height*3 bytes (write-color!'s 0..255 values) -> PNG file."
  [path ^bytes rgb width height]
  (Native/writePng (str path) rgb (int width) (int height)))

(defn ppm->png
  "src/ppm2png.clj:35-87's ppm->png through the library."
  [source dest]
  (Native/ppmToPng (str source) (str dest)))

;; The reference's five bodies (raytracing.clj:63-78) as data.
(def hittables
  [{:center [0.0 -100.5 -1.0] :radius 100.0 :material {:type :lambertian :albedo [0.8 0.8 0.0]}}
   {:center [0.0 0.0 -1.2] :radius 0.5 :material {:type :lambertian :albedo [0.1 0.2 0.5]}}
   {:center [-1.0 0.0 -1.0] :radius 0.5 :material {:type :dielectric :refraction-index 1.5}}
   {:center [-1.0 0.0 -1.0] :radius 0.4 :material {:type :dielectric :refraction-index (/ 1.0 1.5)}}
   {:center [1.0 0.0 -1.0] :radius 0.5 :material {:type :metal :albedo [0.8 0.6 0.2] :fuzz 1.0}}])

(defn -main
  "`clojure -M:main [spp] [depth]` (raytracing.clj:95-177) on the GPU: the
  same config line, (time ...) around render + PPM + PNG (scene.ppm, then
  ppm->png to scene.png inside the timing, as raytracing.clj:176 does)."
  [& args]
  (let [spp (if (first args) (Integer/parseInt (first args)) 100)
        depth (if (second args) (Integer/parseInt (second args)) 50)
        width 400
        height (int (/ width 16/9))]
    (println "config:" {:samples-per-px spp :max-depth depth})
    (time
     (let [cam (camera width height {:vfov 20.0 :look-from [-2.0 2.0 1.0] :look-at [0.0 0.0 -1.0]
                                     :vup [0.0 1.0 0.0] :defocus-angle 10.0 :focus-dist 3.4})
           rgb (render-bytes hittables cam {:width width :height height :samples-per-px spp :max-depth depth})]
       (write-ppm! "scene.ppm" rgb width height)
       (ppm->png "scene.ppm" "scene.png")))))
