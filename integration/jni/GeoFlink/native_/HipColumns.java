/*
 * HipColumns -- the SoA hand-over the window functions share: a window's Points copied into
 * direct ByteBuffers (native order; x, y: double, objID keys: long) that the natives read, and
 * GeoFlink Polygons flattened into the CSR arrays the polygon natives take.  NOT COMPILED here
 * (no JDK in the build image); see INTEGRATION.md.
 *
 * Polygons: ringOff[npoly + 1] indexes rings, vertOff[nrings + 1] indexes vx / vy; each polygon is
 * its JTS exterior ring then its holes (Polygon.polygon, Polygon.java:22), rings closed as JTS keeps
 * them -- the layout gf_polygons expects (include/geoflink_hip.h).
 */
package GeoFlink.native_;

import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
import org.locationtech.jts.geom.Coordinate;
import org.locationtech.jts.geom.LineString;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;

final class HipColumns {
  ByteBuffer x, y, objID;        // objID only when withObjID
  private final boolean withObjID;
  private String[] ids = new String[0];

  HipColumns(boolean withObjID) { this.withObjID = withObjID; }

  /** the points' x, y (and objID keys, interned in ctx's dictionary) -> the direct buffers */
  void fill(long ctx, List<Point> pts) {
    final int n = pts.size();
    if (x == null || x.capacity() < 8 * n) {
      final int cap = Math.max(1 << 12, n + n / 4);
      x = ByteBuffer.allocateDirect(8 * cap).order(ByteOrder.nativeOrder());
      y = ByteBuffer.allocateDirect(8 * cap).order(ByteOrder.nativeOrder());
      if (withObjID) objID = ByteBuffer.allocateDirect(8 * cap).order(ByteOrder.nativeOrder());
      ids = new String[cap];
    }
    for (int i = 0; i < n; i++) {
      final Point p = pts.get(i);
      x.putDouble(8 * i, p.point.getX());
      y.putDouble(8 * i, p.point.getY());
      if (withObjID) ids[i] = p.objID;
    }
    if (withObjID) {  // Point.objID Strings -> keys (the merges dedupe by String.equals)
      final long[] keys = GeoFlinkHip.intern(ctx, ids, n);
      objID.asLongBuffer().put(keys, 0, n);
    }
  }

  /** a direct int buffer of at least n entries (index lists the natives write) */
  static ByteBuffer ints(ByteBuffer b, long n) {
    if (b != null && b.capacity() >= 4 * n) return b;
    final long cap = Math.max(1 << 12, n + n / 4);
    return ByteBuffer.allocateDirect((int) (4 * cap)).order(ByteOrder.nativeOrder());
  }

  static <T> List<T> list(Iterable<T> it, List<T> into) {
    into.clear();
    for (T t : it) into.add(t);
    return into;
  }

  /** polygons as CSR: {ringOff, vertOff} in ints, {vx, vy} in coords */
  static final class Csr {
    final int[] ringOff, vertOff;
    final double[] vx, vy;

    Csr(Collection<Polygon> polygons) {
      final List<LineString> rings = new ArrayList<>();
      ringOff = new int[polygons.size() + 1];
      int p = 0;
      for (Polygon poly : polygons) {
        final org.locationtech.jts.geom.Polygon g = poly.polygon;
        rings.add(g.getExteriorRing());
        for (int h = 0; h < g.getNumInteriorRing(); h++) rings.add(g.getInteriorRingN(h));
        ringOff[++p] = rings.size();
      }
      vertOff = new int[rings.size() + 1];
      int nv = 0;
      for (int r = 0; r < rings.size(); r++) vertOff[r + 1] = nv += rings.get(r).getNumPoints();
      vx = new double[nv];
      vy = new double[nv];
      int v = 0;
      for (LineString ring : rings)
        for (Coordinate c : ring.getCoordinates()) {
          vx[v] = c.x;
          vy[v++] = c.y;
        }
    }
  }
}
