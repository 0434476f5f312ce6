package io.sesam.dukemicroservice.gpu;

import java.util.List;

import no.priv.garshol.duke.Property;
import no.priv.garshol.duke.Record;
import no.priv.garshol.duke.databases.KeyFunction;

/**
 * A blocking key function with a native form (dk_key_function): the concatenation of parts,
 * each a property's value, optionally one of its whitespace tokens (negative = from the end),
 * sliced [start, end) in code points with Python slice rules -- exactly what dk_pack_json
 * computes for a POSTed body, so a pipeline whose key functions are all PartsKeyFunction can
 * take native ingestion.  Mirrors dukehip.records.PartsKey (a missing value contributes "").
 */
public class PartsKeyFunction implements KeyFunction {
    /** One part: the property, its token (DukeHip.KEY_ALL = the whole value), slice bounds
     *  (DukeHip.KEY_ALL = open end). */
    public static final class Part {
        final String property;
        final int token, start, end;

        public Part(String property, int token, int start, int end) {
            this.property = property;
            this.token = token;
            this.start = start;
            this.end = end;
        }
    }

    private final Part[] parts;

    public PartsKeyFunction(Part... parts) {
        this.parts = parts;
    }

    @Override
    public String makeKey(Record record) {
        StringBuilder sb = new StringBuilder();
        for (Part p : parts) sb.append(part(record.getValue(p.property), p));
        return sb.toString();
    }

    /** dk_key_function parts (prop index into the scored properties, token, start, end)*. */
    public int[] parts(List<Property> scoredProps) {
        int[] out = new int[4 * parts.length];
        for (int i = 0; i < parts.length; i++) {
            int idx = -1;
            for (int k = 0; k < scoredProps.size(); k++)
                if (scoredProps.get(k).getName().equals(parts[i].property)) idx = k;
            if (idx < 0) throw new IllegalArgumentException("key part on an unscored property " + parts[i].property);
            out[4 * i] = idx;
            out[4 * i + 1] = parts[i].token;
            out[4 * i + 2] = parts[i].start;
            out[4 * i + 3] = parts[i].end;
        }
        return out;
    }

    // Python's str.isspace over the BMP: Java's whitespace plus NEL and the no-break spaces
    private static boolean space(int c) {
        return Character.isWhitespace(c) || c == 0x85 || c == 0xA0 || c == 0x2007 || c == 0x202F;
    }

    private static String part(String value, Part p) {
        if (value == null) return "";
        if (p.token != DukeHip.KEY_ALL) {  // str.split(): runs of whitespace, none empty
            List<String> toks = new java.util.ArrayList<>();
            int i = 0, n = value.length();
            while (i < n) {
                while (i < n && space(value.charAt(i))) i++;
                int a = i;
                while (i < n && !space(value.charAt(i))) i++;
                if (i > a) toks.add(value.substring(a, i));
            }
            int t = p.token < 0 ? p.token + toks.size() : p.token;
            value = t >= 0 && t < toks.size() ? toks.get(t) : "";
        }
        int len = value.codePointCount(0, value.length());
        int a = bound(p.start, len, 0), b = bound(p.end, len, len);
        if (b <= a) return "";
        return value.substring(value.offsetByCodePoints(0, a), value.offsetByCodePoints(0, b));
    }

    private static int bound(int v, int len, int open) {
        if (v == DukeHip.KEY_ALL) return open;
        if (v < 0) v += len;
        return Math.max(0, Math.min(v, len));
    }
}
