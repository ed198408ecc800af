/*
 * GeoFlinkHip -- the Java side of the JNI shim that puts libgeoflink_hip.so behind the GeoFlink
 * window operators (see INTEGRATION.md).  NOT COMPILED in this repository: the build image has
 * no JDK (no javac, no jni.h).  It is kept as a real source file so a maintainer can drop it
 * next to the reference's operators (package GeoFlink.native_) and build it with the JDK.
 *
 * Every handle is a native pointer held in a long.  Window buffers are direct ByteBuffers in
 * native byte order (x, y: double; objID, ts: long).  Each plan caches its device window(s), so
 * a continuous query uploads into the same device buffers window after window.
 *
 * Anchors (what each native call replaces):
 *   knnWindow    PointPointKNNQuery.windowBased (PointPointKNNQuery.java:132-201) +
 *                KNNQuery.kNNWinAllEvaluationPointStream (KNNQuery.java:213-272)
 *   rangeWindow  PointPointRangeQuery.windowBased apply (PointPointRangeQuery.java:150-186),
 *                PointPolygonRangeQuery apply (PointPolygonRangeQuery.java:170-204)
 *   joinWindow   JoinQuery.getReplicatedPointQueryStream (JoinQuery.java:73-90) +
 *                PointPointJoinQuery.windowBased (PointPointJoinQuery.java:148-182)
 *   polygonJoinWindow  JoinQuery.java:93-115 + PointPolygonJoinQuery.java:154-213
 *   csvParse     Deserialization.CSVTSVToTSpatial.map (Deserialization.java:291-325)
 *   geoJsonParse Deserialization.GeoJSONToSpatial (Deserialization.java:149-211), Point features
 */
package GeoFlink.native_;

import java.nio.ByteBuffer;

public final class GeoFlinkHip {
  static { System.loadLibrary("geoflink_jni"); }   // libgeoflink_jni.so -> libgeoflink_hip.so

  private GeoFlinkHip() {}

  // one context per Flink subtask (RichAllWindowFunction.open / close)
  public static native long ctxCreate(int device);
  public static native void ctxDestroy(long ctx);

  // ---- kNN (point query) ----------------------------------------------------------------
  // UniformGrid(n, minX, maxX, minY, maxY) is passed by value
  public static native long knnPlan(long ctx, int n, double minX, double maxX, double minY, double maxY,
                                    double qx, double qy, double r, int k);
  public static native void knnPlanDestroy(long plan);
  // x, y, objID of one window (ts is not read by window evaluation); returns the number of
  // neighbours written to out* (ascending (dist, objID)), outIdx = the window-local indices
  public static native int knnWindow(long plan, ByteBuffer x, ByteBuffer y, ByteBuffer objID, int n,
                                     long[] outObjID, double[] outDist, long[] outIdx);

  // ---- range ---------------------------------------------------------------------------
  public static native long rangePlan(long ctx, int n, double minX, double maxX, double minY, double maxY,
                                      double[] qx, double[] qy, double r, boolean approximate);
  // polygons as CSR: ringOff[npoly+1] into vertOff, vertOff[nrings+1] into vx / vy (closed rings)
  public static native long rangePolygonPlan(long ctx, int n, double minX, double maxX, double minY, double maxY,
                                             int[] ringOff, int[] vertOff, double[] vx, double[] vy, double r,
                                             boolean approximate);
  public static native void rangePlanDestroy(long plan);
  // emitted point indices, ascending
  public static native int[] rangeWindow(long plan, ByteBuffer x, ByteBuffer y, int n);

  // ---- joins ---------------------------------------------------------------------------
  // grids as {n, minX, maxX, minY, maxY}; pairs (ordinary index, query index) flattened
  public static native long[] joinWindow(long ctx, double[] uGrid, double[] qGrid, ByteBuffer ox, ByteBuffer oy,
                                         int no, ByteBuffer qx, ByteBuffer qy, int nq, double r,
                                         boolean approximate);
  public static native long[] polygonJoinWindow(long ctx, double[] grid, ByteBuffer x, ByteBuffer y, int n,
                                                int[] ringOff, int[] vertOff, double[] vx, double[] vy, double r,
                                                boolean approximate);

  // ---- ingest --------------------------------------------------------------------------
  // a chunk of complete lines -> x, y, objID keys, ts (direct buffers of capacity >= lines);
  // returns the number of points; objID Strings are interned in the context's dictionary
  public static native int csvParse(long ctx, ByteBuffer text, int len, char delimiter, int[] schema /* objID, ts, x, y */,
                                    ByteBuffer x, ByteBuffer y, ByteBuffer objID, ByteBuffer ts, int capacity);
  // GeoJSON Point features (one per line) -> the same columns
  public static native int geoJsonParse(long ctx, ByteBuffer text, int len, ByteBuffer x, ByteBuffer y,
                                        ByteBuffer objID, ByteBuffer ts, int capacity);
}
