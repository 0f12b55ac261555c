# %% [markdown]
# # Maps with drawing controls (ipyleaflet stand-in)
# Mirrors notebooks/ml/Plotting/ipyleaflet.ipynb:21-251: a map centred on (34.63, -77.35) at zoom 7,
# a DrawControl with marker / rectangle / circle tools and a draw callback, last_action / last_draw,
# clear_* calls, a second map linked on center and zoom, the last drawing added to it as GeoJSON.
# Drawing is an API call here (no browser): it fires the same callback with the same GeoJSON.
# %%
from hops_examples_amd.plotting import DrawControl, GeoJSON, Map, link

center = [34.6252978589571, -77.34580993652344]
zoom = 7
m = Map(center=center, zoom=zoom)
print(m.zoom)

# %%
dc = DrawControl(marker={"shapeOptions": {"color": "#0000FF"}}, rectangle={"shapeOptions": {"color": "#0000FF"}},
                 circle={"shapeOptions": {"color": "#0000FF"}}, circlemarker={})
events = []


def handle_draw(self, action, geo_json):
    print(action)
    print(geo_json)
    events.append(action)


dc.on_draw(handle_draw)
m.add_control(dc)
dc.draw("marker", (34.7, -77.2))
dc.draw("rectangle", ((34.4, -77.6), (34.9, -77.0)))
print(dc.last_action, dc.last_draw["geometry"]["type"])
dc.clear_circles()
dc.clear_markers()
assert [s["properties"]["kind"] for s in dc.shapes] == ["rectangle"]

# %%
m2 = Map(center=center, zoom=zoom, layout=dict(width="600px", height="400px"))
map_center_link = link((m, "center"), (m2, "center"))
map_zoom_link = link((m, "zoom"), (m2, "zoom"))
m.zoom = 9
assert m2.zoom == 9
new_poly = GeoJSON(data=dc.last_draw)
m2.add_layer(new_poly)
dc2 = DrawControl(polygon={"shapeOptions": {"color": "#0000FF"}}, polyline={},
                  circle={"shapeOptions": {"color": "#0000FF"}})
m2.add_control(dc2)
dc2.draw("polygon", [(34.5, -77.5), (34.8, -77.1), (34.4, -77.0)])
m2.add_layer(GeoJSON(data=dc2.last_draw))
print(m2.save("Resources/plots/linked_map.svg"), events)
