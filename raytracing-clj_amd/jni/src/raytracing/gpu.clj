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

(defn render
  "width*height*3 linear RGB floats: compute-pixel's accum/spp for every pixel.
  camera keys are the values -main derives (raytracing.clj:126-139).
  :realm? true renders with realm.raytracing's semantics (RT_FLAG_REALM:
  src/realm/raytracing.clj; pass realm's camera: no defocus, focal length
  |look-from - look-at|)."
  [bodies {:keys [center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v defocus-angle]}
   {:keys [width height samples-per-px max-depth seed gpus realm?] :or {seed 1 gpus 0}}]
  (let [[sph knd mat] (flatten-bodies bodies)
        cam (float-array (concat center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v))
        out (float-array (* width height 3))]
    (Native/renderWithFlags sph knd mat cam (if (pos? (or defocus-angle 0)) 1 0) width height
                            samples-per-px max-depth (long seed) (int gpus)
                            (if realm? Native/FLAG_REALM 0) out)
    out))

(defn write-png!
  "rgb: width*height*3 bytes (write-color!'s 0..255 values) -> PNG file."
  [path ^bytes rgb width height]
  (Native/writePng (str path) rgb (int width) (int height)))

(defn ppm->png
  "src/ppm2png.clj:35-87's ppm->png through the library."
  [source dest]
  (Native/ppmToPng (str source) (str dest)))
