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
  camera keys are the values -main derives (raytracing.clj:126-139)."
  [bodies {:keys [center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v defocus-angle]}
   {:keys [width height samples-per-px max-depth seed gpus] :or {seed 1 gpus 0}}]
  (let [[sph knd mat] (flatten-bodies bodies)
        cam (float-array (concat center pixel-00-loc pixel-du pixel-dv defocus-disk-u defocus-disk-v))
        out (float-array (* width height 3))]
    (Native/render sph knd mat cam (if (pos? defocus-angle) 1 0) width height
                   samples-per-px max-depth (long seed) (int gpus) out)
    out))
